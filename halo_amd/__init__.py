"""halo_amd: MI355X (gfx950) backend for the rasmus-kirk/halo proving hot path.

The compute lives in libhalo_gpu.so (hand-written HIP behind the C ABI of include/halo_gpu.h);
this package is the thin host-side mirror of the reference's Rust surface on that path, with the
reference's names, argument meaning and assertion messages:

    halo_amd.group    -- crates/group/src/group.rs  (scalar_dot, point_dot_affine, construct_powers),
                         crates/group/src/pp.rs     (PublicParams: resident SRS)
    halo_amd.poly     -- crates/group/src/poly.rs   (Domain, Evals: NTT / iNTT wrappers)
    halo_amd.pedersen -- crates/accumulation/src/pedersen.rs (commit)
    halo_amd.pcdl     -- crates/accumulation/src/pcdl.rs     (commit, open_without_eval round loop)

Field elements are numpy uint64 arrays of shape (n, 4) in arkworks Montgomery form; points are
(n, 8) WrappedPoint arrays (x, y Montgomery limbs; (0, 0) = identity).  There is no CPU fallback:
without the HIP library or a GPU every call raises.
"""
from . import _lib  # noqa: F401

__all__ = ["_lib", "group", "poly", "pedersen", "pcdl"]
