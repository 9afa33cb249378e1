"""CPU tests of the C ABI boundary: libgpx.so loads, exports every symbol include/gpx.h declares, the ctypes
structs match the header layout, and the pure host-side queries answer without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from bayesianoptimizer_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_capi.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "bayesianoptimizer_amd", "csrc")], check=True)
    return _capi.load()


def test_library_exports_every_header_symbol(lib):
    syms = _capi.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, f"header declares symbols the library does not export: {missing}"
    # and the ctypes prototypes cover exactly the header
    assert sorted(_capi._PROTOS) == syms


def test_exported_symbols_are_plain_c(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (gpx_[a-z0-9_]+)\b", out))
    assert set(_capi.header_symbols()) <= exported  # unmangled extern "C"


def test_version_and_padding(lib):
    assert lib.gpx_version().decode().startswith("gpx ")
    for n, p in [(1, 128), (128, 128), (129, 256), (4096, 4096), (16384, 16384), (4097, 4224)]:
        assert lib.gpx_padded_n(n) == p


def test_loaded_library_is_built_from_this_tree(lib):
    """Binary provenance: the Makefile stamps a sha256 of csrc/* + include/gpx.h into gpx_version();
    the library the tests load must carry the hash of the working tree's sources, not an A/B or stale build."""
    assert _capi.library_source_sha256(lib) == _capi.source_sha256(), lib.gpx_version().decode()



def test_struct_layout_matches_header():
    # gpx_kernel_params: 2 int32 + 2*32 doubles + 4 doubles + 2 int32
    assert ctypes.sizeof(_capi.KernelParamsC) == 8 + 2 * 32 * 8 + 4 * 8 + 8
    assert _capi.KernelParamsC.cov_fp32.offset == 8 + 2 * 32 * 8 + 4 * 8
    assert _capi.KernelParamsC.lengthscale.offset == 8
    assert _capi.KernelParamsC.outputscale.offset == 8 + 2 * 32 * 8
    assert ctypes.sizeof(_capi.AcqParamsC) == 8 + 4 * 8
    hdr = open(_capi.HEADER_PATH).read()
    assert "#define GPX_MAX_DIM 32" in hdr and "#define GPX_MAX_RHS 8" in hdr and "#define GPX_TILE 128" in hdr


def test_header_constants_match_python():
    hdr = open(_capi.HEADER_PATH).read()
    for name, val in [("GPX_OK", 0), ("GPX_NOT_PD", 1), ("GPX_INVALID_ARG", 2), ("GPX_HIP_ERROR", 3),
                      ("GPX_KERNEL_RBF", 0), ("GPX_KERNEL_MATERN52", 1), ("GPX_KERNEL_SCALE_LINEAR_MATERN52", 2),
                      ("GPX_ACQ_EI", 0), ("GPX_ACQ_LOGEI", 1), ("GPX_ACQ_UCB", 2), ("GPX_ACQ_VARIANCE", 3),
                      ("GPX_TIMER_TRMM", 5)]:
        assert re.search(rf"\b{name} = {val}\b", hdr), name
    # the per-handle option numbering the binding uses: stable ABI numbers, the removed potrf_schedule keeps slot 0 as
    # GPX_OPT_RESERVED_0 (round 4 had renumbered the enum without an ABI bump)
    for name, val in _capi.OPTIONS.items():
        assert re.search(rf"\bGPX_OPT_{name.upper()} = {val}\b", hdr), name
    assert _capi.OPTIONS["spin_limit"] == 1 and _capi.OPTIONS["potrf_mode"] == 5
    assert re.search(r"\bGPX_OPT_RESERVED_0 = 0\b", hdr)
    assert re.search(rf"\bGPX_OPT_COUNT = {_capi.GPX_OPT_COUNT}\b", hdr)


def test_workspace_queries_without_gpu(lib):
    b = ctypes.c_size_t()
    assert lib.gpx_fit_workspace_size(4096, 1, ctypes.byref(b)) == _capi.GPX_OK
    assert b.value >= 4096 * 4096 // 4 * 8
    assert lib.gpx_sweep_workspace_size(4096, 1, 1 << 20, ctypes.byref(b)) == _capi.GPX_OK
    assert b.value >= 4096 * 8192 * 8  # one K* chunk
    assert lib.gpx_sweep_workspace_size(4096, 9, 10, ctypes.byref(b)) == _capi.GPX_INVALID_ARG
    assert lib.gpx_alpha_workspace_size(0, 1, ctypes.byref(b)) == _capi.GPX_INVALID_ARG
    assert lib.gpx_trtri_workspace_size(100, None) == _capi.GPX_INVALID_ARG
    one = ctypes.c_size_t()
    assert lib.gpx_fit_workspace_size(4096, 1, ctypes.byref(one)) == _capi.GPX_OK
    assert lib.gpx_fit_batched_workspace_size(4096, 1, 4, ctypes.byref(b)) == _capi.GPX_OK
    assert b.value >= 4 * one.value  # one workspace slice per problem
    assert lib.gpx_fit_batched_workspace_size(4096, 1, 0, ctypes.byref(b)) == _capi.GPX_INVALID_ARG


def test_null_handle_is_rejected(lib):
    assert lib.gpx_destroy(None) == _capi.GPX_INVALID_ARG
    assert lib.gpx_set_stream(None, None) == _capi.GPX_INVALID_ARG
    assert lib.gpx_last_error(None) == b"invalid handle"
    assert lib.gpx_timing_enable(None, 1) == _capi.GPX_INVALID_ARG


def test_engine_refuses_cpu_device():
    import torch

    from bayesianoptimizer_amd import GPEngine

    with pytest.raises(ValueError):
        GPEngine(torch.device("cpu"))


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_capi, "_lib", None)
    monkeypatch.setattr(_capi, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_capi.GPXLibraryError):
        _capi.load()


def _integration_struct():
    """The KernelParams class of INTEGRATION.md's ctypes binding snippet, executed as documented."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.search(r"```python\n(# optimization/gpx_binding\.py.*?)```", text, re.S).group(1)
    start = block.index("class KernelParams(ctypes.Structure):")
    cls = block[start:block.index("\n\n", start)]
    ns = {"ctypes": ctypes}
    exec(cls, ns)  # noqa: S102 - our own documentation
    assert "assert ctypes.sizeof(KernelParams) == lib.gpx_kernel_params_size()" in block
    return ns["KernelParams"]


def test_integration_binding_struct_matches_header(lib):
    doc = _integration_struct()
    assert ctypes.sizeof(doc) == ctypes.sizeof(_capi.KernelParamsC) == lib.gpx_kernel_params_size() == 560
    assert [f[0] for f in doc._fields_] == [f[0] for f in _capi.KernelParamsC._fields_]
    for name, _ in _capi.KernelParamsC._fields_:
        assert getattr(doc, name).offset == getattr(_capi.KernelParamsC, name).offset, name
        assert getattr(doc, name).size == getattr(_capi.KernelParamsC, name).size, name
    assert lib.gpx_acq_params_size() == ctypes.sizeof(_capi.AcqParamsC) == 40


def test_truncated_struct_binding_is_refused(monkeypatch):
    """A binding whose gpx_kernel_params stops before cov_fp32/reserved (the 552-byte struct of round 1's doc) is
    refused at load instead of letting the library read past the caller's object."""
    class Truncated(ctypes.Structure):
        _fields_ = _capi.KernelParamsC._fields_[:-2]

    assert ctypes.sizeof(Truncated) == 552
    monkeypatch.setattr(_capi, "_lib", None)
    monkeypatch.setattr(_capi, "KernelParamsC", Truncated)
    with pytest.raises(_capi.GPXLibraryError, match="552 bytes, libgpx expects 560"):
        _capi.load()
    monkeypatch.undo()
    _capi._lib = None
    _capi.load()
