// Runtime field / curve id -> template type dispatch.
#pragma once
#include "curve.hpp"

#define DISPATCH_FIELD(fid, T, ...)        \
    do {                                   \
        if ((fid) == HALO_FP) {            \
            using T = ::halo::FpCfg;       \
            __VA_ARGS__;                   \
        } else {                           \
            using T = ::halo::FqCfg;       \
            __VA_ARGS__;                   \
        }                                  \
    } while (0)

#define DISPATCH_CURVE(cid, T, ...)        \
    do {                                   \
        if ((cid) == HALO_PALLAS) {        \
            using T = ::halo::PallasCurve; \
            __VA_ARGS__;                   \
        } else {                           \
            using T = ::halo::VestaCurve;  \
            __VA_ARGS__;                   \
        }                                  \
    } while (0)
