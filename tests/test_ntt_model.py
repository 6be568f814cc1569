"""CPU check of the NTT pass kernel's dataflow and limb bounds (tools/ntt_model.py).

The model replays one workgroup of halo_amd/csrc/ntt.hip k_ntt_pass thread by thread -- positions,
thread orders (the wave-uniform unit-twiddle groups of ntt_unit_tau), the alternation of partial and
full normalizations -- with the exact limb arithmetic of the signed lazy butterflies, asserts every
bound the kernel relies on (int32 limbs, fs_mul operands within +-3 x 2^29, fs_settle inputs within
+-4 x 2^29) and compares the block's outputs with a direct DFT.  The GPU tests (test_gpu_ntt.py) run
the kernel itself against the C oracle.
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import ntt_model  # noqa: E402


@pytest.mark.parametrize("NE,r,T,kw", [
    (2048, 11, 1, {}),                      # 2^21 / 2^22 passes: G0 = 1 (no unit group since round 6)
    (2048, 11, 1, {"out_mul": True}),       # ... last pass whose output path multiplies
    (2048, 11, 1, {"prune": 3}),            # ... zero-tail first pass
    (2048, 10, 2, {"pretwiddle": True}),    # 2^20 passes
    (2048, 9, 4, {}),
    (1024, 8, 4, {"pretwiddle": True}),     # 2^23 / 2^24 passes: unit group at stage 2
    (1024, 7, 8, {"prune": 2}),             # ... odd radix, pruned
    (1024, 3, 128, {}),
])
def test_ntt_block_model(NE, r, T, kw):
    M = ntt_model.dft_check(NE, r, T, seed=r + T, **kw)
    assert M.max_mul_limb <= 3 * (1 << 29)
