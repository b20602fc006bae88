"""ctypes binding of the C-ABI library ``libcmx_hip.so``.

The argument/return types are derived by parsing ``include/cmx_hip.h`` (shipped inside
the package as ``cmx_hip.h``), so the header is the single source of truth for the ABI.

The library is loaded AFTER ``import torch`` so that its ``libamdhip64.so.7`` dependency
resolves (by SONAME) to the HIP runtime torch already loaded: kernels then run on torch's
streams and are captured by torch's HIP graphs.  There is no fallback: if the library is
missing or fails to load, importing the product raises.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# CMX_LIB_VARIANT=name loads libcmx_hip_<name>.so (an A/B build of the same sources with other
# compile-time options, csrc/Makefile VARIANT=); default: libcmx_hip.so
_VARIANT = os.environ.get("CMX_LIB_VARIANT", "")
LIB_PATH = os.path.join(_HERE, f"libcmx_hip_{_VARIANT}.so" if _VARIANT else "libcmx_hip.so")
HEADER_PATHS = [os.path.join(_HERE, "..", "include", "cmx_hip.h"), os.path.join(_HERE, "cmx_hip.h")]


class CMXError(RuntimeError):
    pass


# cmx_status codes (csrc/cmx_common.h)
CMX_OK, CMX_ERR_SHAPE, CMX_ERR_DTYPE, CMX_ERR_LAUNCH, CMX_ERR_ARG = 0, -1, -2, -3, -4


def _ctype(decl: str):
    decl = decl.strip()
    if "*" in decl:
        if decl.startswith("const char") and decl.count("*") == 1 and not decl.split("*")[1].strip():
            return ctypes.c_char_p
        return ctypes.c_void_p
    base = decl.rsplit(" ", 1)[0] if " " in decl else decl
    base = base.replace("const", "").strip()
    return {"int": ctypes.c_int32, "int64_t": ctypes.c_int64, "uint64_t": ctypes.c_uint64, "float": ctypes.c_float,
            "size_t": ctypes.c_size_t, "double": ctypes.c_double, "hipStream_t": ctypes.c_void_p, "void": None}[base]


def parse_header(path: str | None = None):
    """Return {name: (restype, [argtypes])} for every declaration in cmx_hip.h."""
    if path is None:
        path = next(p for p in HEADER_PATHS if os.path.exists(p))
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*([A-Za-z_][\w\s\*]*?)\b(cmx_\w+)\s*\(([^)]*)\)\s*;", text, re.M):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        rt = _ctype(ret.strip() + " r") if "*" not in ret else _ctype(ret.strip() + " r")
        if ret.strip() == "const char*":
            rt = ctypes.c_char_p
        argt = [] if args in ("", "void") else [_ctype(a) for a in args.split(",")]
        out[name] = (rt, argt)
    return out


def header_abi_version(path: str | None = None) -> int:
    """The CMX_ABI_VERSION the header defines (the revision the bindings below are parsed from)."""
    if path is None:
        path = next(p for p in HEADER_PATHS if os.path.exists(p))
    m = re.search(r"^#define\s+CMX_ABI_VERSION\s+(\d+)", open(path).read(), re.M)
    if m is None:
        raise CMXError(f"{path} defines no CMX_ABI_VERSION")
    return int(m.group(1))


def _load():
    if not os.path.exists(LIB_PATH):
        raise CMXError(f"libcmx_hip.so not found at {LIB_PATH}; run __graft_entry__.build() "
                       "(or `make -C rgbx_semantic_segmentation_amd/csrc`).  There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    lib.cmx_abi_version.restype = ctypes.c_int32
    lib.cmx_abi_version.argtypes = []
    want, have = header_abi_version(), int(lib.cmx_abi_version())
    if have != want:
        raise CMXError(f"{LIB_PATH} was built for C-ABI revision {have}, the header declares {want}: "
                       "rebuild it (`make -C rgbx_semantic_segmentation_amd/csrc`)")
    sigs = parse_header()
    for name, (rt, argt) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = rt
    return lib, sigs


LIB, SIGNATURES = _load()


def last_error() -> str:
    return LIB.cmx_last_error().decode()


# measurement hook (roofline.measure_gemm_family): observer(name, fn, args) runs right after a
# successful call, while the caller still holds every buffer the arguments point to
observer = None


def call(name: str, *args) -> None:
    """Invoke an int-returning entry point; raise CMXError on a negative status."""
    fn = getattr(LIB, name)
    st = fn(*args)
    if st != 0:
        raise CMXError(f"{name} failed ({st}): {last_error()}")
    if observer is not None:
        observer(name, fn, args)


def try_call(name: str, *args) -> int:
    """Invoke an int-returning entry point and return its status (the caller decides what a
    refusal means); the measurement observer sees it only when it succeeded."""
    fn = getattr(LIB, name)
    st = int(fn(*args))
    if st == 0 and observer is not None:
        observer(name, fn, args)
    return st


def query(name: str, *args) -> int:
    return int(getattr(LIB, name)(*args))


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float16:
        return 2
    raise CMXError(f"unsupported dtype {t.dtype}")
