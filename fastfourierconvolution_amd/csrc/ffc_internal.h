// Internal helpers shared by the gfx950 kernels of the FFC hot path.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ffc_amd.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace ffc {

void set_error(const std::string& msg);
int launch_status(const char* what);  // FFC_OK or FFC_E_LAUNCH after checking hipGetLastError

#define FFC_CHECK_ARG(cond, msg)              \
    do {                                      \
        if (!(cond)) {                        \
            ::ffc::set_error(msg);            \
            return FFC_E_INVALID;             \
        }                                     \
    } while (0)

__device__ __forceinline__ float apply_act(float v, int act, float p) {
    switch (act) {
        case FFC_ACT_RELU: return fmaxf(v, 0.0f);
        case FFC_ACT_LEAKY_RELU: return v > 0.0f ? v : v * p;
        case FFC_ACT_TANH: return tanhf(v);
        case FFC_ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
        case FFC_ACT_GELU: return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
        default: return v;
    }
}

// Sum over the 32 lanes of each half-wave (lanes l and l^k, k < 32).
__device__ __forceinline__ float half_wave_sum(float v) {
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace ffc
