"""CPU tests of the drop-in boundary: libhalo_gpu.so loads, exports every symbol include/halo_gpu.h
declares, its host-only helpers work, and every compute entry point fails loudly (no CPU fallback)
when no GPU is visible."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from halo_amd import _lib as H

HEADER = H.HEADER_PATH


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(halo_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib_path():
    if not os.path.exists(H.LIB_PATH):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(os.path.dirname(H.LIB_PATH), "..", "csrc")], check=True)
    return H.LIB_PATH


def test_header_declares_expected_surface():
    syms = declared_symbols()
    for s in ("halo_msm", "halo_pcdl_commit", "halo_ntt", "halo_interpolate", "halo_ipa_fold", "halo_poly_eval_batch"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib_path):
    L = ctypes.CDLL(lib_path)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert missing == []


def test_python_binding_covers_header(lib_path):
    assert sorted(H.SIGNATURES) == declared_symbols()
    assert H.missing_symbols(lib_path) == []


def test_library_is_gfx950_code(lib_path):
    data = open(lib_path, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_synth_scalar_host_function(lib_path):
    from halo_amd.group import synth_scalar
    a = synth_scalar(7, 0)
    b = synth_scalar(7, 0)
    c = synth_scalar(7, 1)
    assert a == b != c
    assert 0 < a < (1 << 253)


def test_abi_version(lib_path):
    assert H.load().halo_abi_version() >= 100


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and H.load().halo_device_count() > 0,
                    reason="a GPU is visible")
def test_fails_loudly_without_gpu(lib_path):
    L = H.load()
    x = np.zeros((8, 4), dtype=np.uint64)
    rc = L.halo_ntt(0, H.ptr(x), 3, 0)
    assert rc == 3  # HALO_EDEVICE
    assert "device" in H.last_error().lower()
    with pytest.raises(H.HaloError):
        H.ensure_device(0)


def test_tuning_keys_roundtrip_and_reject_unknown(lib_path):
    """halo_set_tuning / halo_get_tuning are host-only: every key round-trips, -1 restores the
    default, an unknown key is HALO_EINVAL (no GPU needed)."""
    defaults = {"ipa_weighted": 1, "ipa_tail": 1, "ipa_srs_tail_n": 4096, "ipa_mat_n": 2048, "msm_multi_max": 1 << 18,
                "ipa_pool_keep_bytes": 1 << 30}
    for k, v in defaults.items():
        assert H.get_tuning(k) == v
        with H.tuning(**{k: 7}):
            assert H.get_tuning(k) == 7
        assert H.get_tuning(k) == v
        H.set_tuning(k, 3)
        H.set_tuning(k, -1)
        assert H.get_tuning(k) == v
    with pytest.raises(H.HaloError):
        H.set_tuning("no_such_key", 1)


def test_library_reads_no_environment():
    """The product library's path selections are the tuning ABI, not environment variables (VERDICT
    r03 item 7): no getenv / secure_getenv in the sources of libhalo_gpu.so (the Python mirror's
    HALO_LIB, used by A/B tools to pick a build, is outside the library)."""
    import glob
    here = os.path.dirname(os.path.abspath(__file__))
    srcs = glob.glob(os.path.join(here, "..", "halo_amd", "csrc", "*.hip")) + \
        glob.glob(os.path.join(here, "..", "halo_amd", "csrc", "*.cpp")) + \
        glob.glob(os.path.join(here, "..", "halo_amd", "csrc", "*.hpp"))
    assert srcs
    for f in srcs:
        text = open(f).read()
        assert not re.search(r"\b(secure_)?getenv\s*\(", text), f
