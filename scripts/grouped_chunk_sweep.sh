cd "${GRAFT_REPO_ROOT}"
timeout -k 10 120 python -u -m pytest tests/test_gpu_grouped.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gc.log 2>&1 || exit 1
for c in ${CHUNKS:-0 4 16 64}; do CMX_GROUPED_CHUNK=$c timeout -k 10 100 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk', $c, d['value'], d['roofline']['avg_launch_us'])" || exit 1; done
