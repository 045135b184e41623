"""CPU tests of the drop-in boundary: libmvc_hip.so loads, exports every entry
point include/mvc.h declares, and rejects bad arguments / a missing GPU with
a status code and a message instead of crashing (no compute without a GPU).
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mvc.h")
PKG = os.path.join(ROOT, "multiview-clustering_amd")


@pytest.fixture(scope="module")
def lib():
    from mvc_amd import _lib as L
    if not os.path.exists(L.LIB_PATH):
        subprocess.run(["make", "-s", "-C", ROOT, "-j8"], check=True)
    return L


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mvc_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = _declared_functions()
    for must in ("mvc_run", "mvc_result_free", "mvc_sampler_create", "mvc_sampler_sweep", "mvc_sampler_get_state",
                 "mvc_sampler_set_state", "mvc_sampler_destroy"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    so = ctypes.CDLL(lib.LIB_PATH)
    missing = [f for f in _declared_functions() if not hasattr(so, f)]
    assert not missing, missing


def test_abi_version_and_defaults(lib):
    L = lib.lib()
    assert L.mvc_abi_version() == 2
    cfg = lib.Config()
    L.mvc_config_init(ctypes.byref(cfg))
    assert cfg.thin >= 1 and cfg.n_chains == 1 and cfg.mode == lib.MODE_EXACT
    assert cfg.n_devices == 0 and cfg.chain_stride == 0   # one device; chain ids first_chain + c


def test_config_layout_matches_header(lib, tmp_path):
    """The ctypes mirror of mvc_config has the C header's size and offsets
    (the Rcpp drop-in carries the same layout)."""
    fields = [f for f, _ in lib.Config._fields_]
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mvc.h"\nint main(void){printf("%zu",'
                   'sizeof(mvc_config));' + "".join(f'printf(" %zu", offsetof(mvc_config, {f}));' for f in fields) +
                   "return 0;}\n")
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got[0] == ctypes.sizeof(lib.Config)
    assert got[1:] == [getattr(lib.Config, f).offset for f in fields]


def test_shard_callback_returns_a_status(lib):
    """mvc_sampler_set_shard's all_gather returns int (0 = done; nonzero fails
    the sweep with MVC_ERR_CALLBACK before the exchange buffer is read)."""
    assert lib.SHARD_CB._restype_ is ctypes.c_int
    assert "int (*all_gather)(void *)" in open(HEADER).read()


def test_loaders_leave_the_hardware_queues_alone(lib):
    """The chain-batched repair needs no hardware queue per chain: neither the
    Python loader nor the Rcpp drop-in sets GPU_MAX_HW_QUEUES any more."""
    import subprocess
    import sys
    code = ("import os, sys; sys.path[:0] = [%r, %r]; os.environ.pop('GPU_MAX_HW_QUEUES', None); "
            "import mvc_amd; mvc_amd.lib(); print(os.environ.get('GPU_MAX_HW_QUEUES'))" % (ROOT, PKG))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().splitlines()[-1] == "None", r.stderr[-800:]
    src = open(os.path.join(PKG, "R", "multiview_gibbs.cpp")).read()
    assert 'setenv("GPU_MAX_HW_QUEUES"' not in src


def _call_run(lib, cfg, y):
    from mvc_amd.sampler import _view_ptrs
    res = ctypes.c_void_p()
    buf = lib.errbuf()
    st = lib.lib().mvc_run(ctypes.byref(cfg), _view_ptrs(y), ctypes.byref(res), buf, len(buf))
    return st, buf.value.decode(), res


@pytest.mark.parametrize("field,value,needle", [
    ("n", 1, "n must be"), ("n_views", 0, "n_views"), ("dim", 0, "dim"), ("thin", 0, "thin"),
    ("n_chains", 0, "n_chains"), ("mode", 7, "mode"), ("n_iter", -1, "n_iter"),
    ("n_devices", -1, "n_devices"), ("chain_stride", -2, "chain_stride"),
])
def test_invalid_config_is_rejected_before_touching_a_device(lib, field, value, needle):
    from mvc_amd.sampler import make_config
    y = np.zeros((2, 10, 1))
    cfg = make_config(10, 2, 1, M=3)
    setattr(cfg, field, value)
    st, msg, res = _call_run(lib, cfg, y)
    assert st == lib.MVC_OK + 1 and needle in msg    # MVC_ERR_ARG
    assert not res.value


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and os.path.exists("/dev/kfd") and
                    os.access("/dev/kfd", os.R_OK), reason="a GPU may be visible here")
def test_no_device_is_an_error_not_a_crash(lib):
    from mvc_amd.sampler import make_config
    y = np.random.default_rng(0).normal(size=(2, 50, 1))
    cfg = make_config(50, 2, 1, M=2)
    st, msg, res = _call_run(lib, cfg, y)
    assert st != lib.MVC_OK and msg
    with pytest.raises(lib.MvcError):
        from mvc_amd import Sampler
        Sampler(y, seed=1, mode="parallel")


def test_product_path_never_imports_the_oracle():
    """The product package must not reference oracle/ (test infrastructure)."""
    pkg = os.path.join(ROOT, "multiview-clustering_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "from oracle" not in text and "import oracle" not in text and "mvo_" not in text, f


def test_c_abi_example_compiles():
    """The plain-C caller (dlopen path of the Rcpp drop-in) builds with gcc."""
    import shutil
    import tempfile
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-o",
                        os.path.join(d, "ex"), os.path.join(ROOT, "examples", "mvc_abi_example.c"), "-ldl"],
                       check=True)


def test_rcpp_dropin_compiles():
    """The Rcpp drop-in (multiview-clustering_amd/R/multiview_gibbs.cpp) is
    compile-checked against a declarations-only stub of the Rcpp API subset
    it uses (tests/rcpp_stub/Rcpp.h; R and Rcpp are absent here)."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([gxx, "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(root, "tests", "rcpp_stub"),
                        os.path.join(root, "multiview-clustering_amd", "R", "multiview_gibbs.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
