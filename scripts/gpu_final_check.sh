#!/bin/bash
# end-of-round check of the committed tree: smoke, the GPU suite, one bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final.log; grep -E "^FAILED" gpurun_out/pytest_final.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py 2>/dev/null | cut -c1-200
