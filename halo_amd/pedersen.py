"""Mirror of crates/accumulation/src/pedersen.rs on the MI355X backend."""
from __future__ import annotations

import numpy as np

from . import _lib as H
from .group import _curve


def commit(w, Gs, ms, curve="pallas") -> np.ndarray:
    """pedersen.rs:7-27: ``assert!(Gs.len() >= ms.len())``, MSM(Gs, ms), plus S * w when w is given
    (S from the resident SRS).  Returns the canonical affine WrappedPoint."""
    H.ensure_device()
    Gs, ms = H.point_array(Gs), H.fe_array(ms)
    wa = H.fe_array(w, 1) if w is not None else None
    out = np.zeros(8, dtype=np.uint64)
    H.check(H.load().halo_pedersen_commit(_curve(curve), H.ptr(wa), H.ptr(Gs), len(Gs), H.ptr(ms), len(ms),
                                          H.ptr(out)))
    return out
