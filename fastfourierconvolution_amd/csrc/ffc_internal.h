// Internal helpers shared by the gfx950 kernels of the FFC hot path.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ffc_amd.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---- fp32-accurate products on the bf16 MFMA (the SPLIT kernel instantiations)
// An fp32 value a splits EXACTLY into three bf16 pieces by truncation: hi = top 8 significand bits,
// mid = the next 8 of a - hi, lo = a - hi - mid (<= 8 significant bits left, so exact in bf16; bf16
// has fp32's exponent range).  a*b = sum of the 9 piece products; the 6 with piece order <= 2 are
// kept (dropped terms < 2^-21 |a b|, the order of fp32 accumulation rounding), each product of two
// bf16 pieces is exact in the fp32 accumulator.  6 x v_mfma_f32_32x32x16_bf16 (32 cycles each) per
// 16 k replace 8 x v_mfma_f32_32x32x2_f32 (64 cycles each): 192 vs 512 MFMA cycles.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Split3 {
    bf16x8 hi, mid, lo;
};

static __device__ __forceinline__ unsigned pack_hi16(unsigned lo_elem, unsigned hi_elem) {
    return __builtin_amdgcn_perm(hi_elem, lo_elem, 0x07060302u);   // {lo_elem[31:16], hi_elem[31:16]}
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

static __device__ __forceinline__ Split3 split3(const float (&v)[8]) {
    u32x4 hv, mv, lv;
#ifndef FFC_SPLIT_PACKED
    // scalar v_sub_f32: packed f32 VALU (v_pk_add_f32) costs extra issue cycles beside MFMAs
    // (MI355X_MICROARCH.md issue-cost rows), and the staging / split code runs beside the MFMA
    // waves on the same SIMD.  Same operations, bit-identical pieces; FFC_SPLIT_PACKED: the old form.
    // Same-box A/B (profiles/r03/s2e): gen64 0.4775 -> 0.4678 ms, fgan128 15.88 -> 15.50 ms, gan64train
    // 10.22 -> 9.97 ms.
    // (A whole-library -fno-slp-vectorize build was faster still but broke the B = 8 generator smoke
    // test -- profiles/r03/s2f -- so the library keeps the default vectorizer.)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        unsigned u[2], u1[2], u2[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float a = v[2 * q + e];
            u[e] = __builtin_bit_cast(unsigned, a);
            const float r1 = a - __builtin_bit_cast(float, u[e] & 0xFFFF0000u);
            u1[e] = __builtin_bit_cast(unsigned, r1);
            const float r2 = r1 - __builtin_bit_cast(float, u1[e] & 0xFFFF0000u);
            u2[e] = __builtin_bit_cast(unsigned, r2);
        }
        hv[q] = pack_hi16(u[0], u[1]);
        mv[q] = pack_hi16(u1[0], u1[1]);
        lv[q] = pack_hi16(u2[0], u2[1]);
    }
#else
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // element pairs: the subtractions as v_pk_add_f32 (FFC_SPLIT_PACKED)
        const f32x2 a = {v[2 * q], v[2 * q + 1]};
        const u32x2 ua = __builtin_bit_cast(u32x2, a);
        const f32x2 r1 = a - __builtin_bit_cast(f32x2, ua & 0xFFFF0000u);
        const u32x2 u1 = __builtin_bit_cast(u32x2, r1);
        const f32x2 r2 = r1 - __builtin_bit_cast(f32x2, u1 & 0xFFFF0000u);
        const u32x2 u2 = __builtin_bit_cast(u32x2, r2);
        hv[q] = pack_hi16(ua[0], ua[1]);
        mv[q] = pack_hi16(u1[0], u1[1]);
        lv[q] = pack_hi16(u2[0], u2[1]);
    }
#endif
    Split3 s;
    s.hi = __builtin_bit_cast(bf16x8, hv);
    s.mid = __builtin_bit_cast(bf16x8, mv);
    s.lo = __builtin_bit_cast(bf16x8, lv);
    return s;
}

static __device__ __forceinline__ floatx16 mfma_split3(const Split3& a, const Split3& b, floatx16 acc) {
    // smallest terms first
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.lo, b.hi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.lo, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.mid, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.hi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.mid, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.hi, acc, 0, 0, 0);
    return acc;
}


namespace ffc {

// Bounds-checked loads through a buffer descriptor: an out-of-range byte offset returns 0, so a
// masked element is a load at offset OOB instead of `ok ? p[i] : 0`, which hipcc compiles into a
// branch around the load and a wait per element.  The base (and size) must be wave-uniform.
constexpr unsigned OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, unsigned long long nbytes) {
    const int n = nbytes >= 0x7FFFFFFFull ? 0x7FFFFFFF : (int)nbytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, n, 0x00020000);
}
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ floatx4 buf_ld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

void set_error(const std::string& msg);
int launch_status(const char* what);  // FFC_OK or FFC_E_LAUNCH after checking hipGetLastError
// the training path's planar 2-D real transforms on the fu2d line FFTs (fu2d_kernels.hip): square
// power-of-two planes up to 128; return 1 when the plane is not handled there (direct DFT instead)
int fft_planes_r2c(const float* x, int P, int H, int W, float iscale, float* Z, void* stream);
int fft_planes_c2r(const float* Z, int P, int H, int W, float iscale, const float* addend, float* y, void* stream);

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
// Sum over each 32-lane half of the wave, in every lane: DPP butterflies inside the 16-lane rows
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: VALU, no LDS) and one
// v_permlane16_swap across the rows of a half (gfx950).  Symmetric steps: all 32 lanes hold the
// bit-identical sum.  (xor __shfl chains compile to ds_bpermute: an LDS round trip per step.)
template <int CTRL>
__device__ __forceinline__ float dpp_full(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float half_wave_sum(float v) {
    v += dpp_full<0xB1>(v);
    v += dpp_full<0x4E>(v);
    v += dpp_full<0x141>(v);
    v += dpp_full<0x140>(v);
    const int iv = __builtin_bit_cast(int, v);
    const auto sw = __builtin_amdgcn_permlane16_swap(iv, iv, false, false);
    return __builtin_bit_cast(float, (int)sw[0]) + __builtin_bit_cast(float, (int)sw[1]);
}

// DPP lane moves (no LDS round trip).  CTRL: 0x111..0x11F row_shr:1..15, 0xB1 quad_perm [1,0,3,2]
// (= lane ^ 1).  Lanes whose source is outside the row read 0 (bound_ctrl).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// Sum over each 16-lane DPP row; the result is valid in lane 15 of the row (inclusive scan).
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_f<0x111>(v);
    v += dpp_f<0x112>(v);
    v += dpp_f<0x114>(v);
    v += dpp_f<0x118>(v);
    return v;
}

// Chan partials of every row of a v_mfma_f32_32x32x2f32 accumulator tile over its first nv
// (1..32) columns, without cross-lane shuffle chains: the tile goes through this wave's LDS
// scratch (32 x 33 floats, conflict-free both ways) and lane pair (2o, 2o+1) reduces row o
// (16 columns each).  Accumulator layout: lane l, register r -> row (r&3) + 8(r>>2) + 4(l>>5),
// column l&31.  Row o = lane >> 1's {mean, M2} are valid in the even lane of the pair.
constexpr int TILE_SCRATCH = 32 * 33;
__device__ __forceinline__ void tile_row_stats(const floatx16& acc, int nv, float* scratch, float& mean, float& m2) {
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int r = 0; r < 16; ++r) scratch[((r & 3) + 8 * (r >> 2) + 4 * h) * 33 + col] = acc[r];
    // same-wave LDS write -> read: the LDS serves a wave's instructions in order
    const int o = lane >> 1, c0 = (lane & 1) * 16;
    float v[16];
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        v[j] = scratch[o * 33 + c0 + j];
        if (c0 + j < nv) s += v[j];
    }
    mean = (s + dpp_f<0xB1>(s)) / (float)nv;
    float q = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float d = v[j] - mean;
        if (c0 + j < nv) q = fmaf(d, d, q);
    }
    m2 = q + dpp_f<0xB1>(q);
}

// LDS-DMA copy of n4 16-byte groups from 16-byte aligned global memory into LDS by whole 64-lane
// wave instructions (global_load_lds_dwordx4; lane i of an instruction lands at dst + 16 i bytes):
// dst needs room for n4 rounded up to 64 groups.  Completion: the issuing waves' vmcnt -- call
// dma_wait() before the barrier after which other waves read dst.
__device__ __forceinline__ void dma_copy16(const float* src, float* dst, int n4, int tid, int nthreads) {
    typedef __attribute__((address_space(1))) void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    for (int i0 = 0; i0 < n4; i0 += nthreads) {
        const int wbase = i0 + (tid & ~63);
        if (wbase < n4) {
            const int i = min(i0 + tid, n4 - 1);   // tail lanes repeat the last group inside the padding
            __builtin_amdgcn_global_load_lds((gptr_t)(src + 4 * (size_t)i), (lptr_t)(dst + 4 * wbase), 16, 0, 0);
        }
    }
}

// Retire this wave's LDS-DMA copies (dma_copy16) before the barrier that publishes them to the other
// waves: LDS-DMA data is ordered for another wave's ds_read only by the issuing wave's vmcnt wait
// followed by a barrier (MI355X_MICROARCH.md item 7).  __syncthreads() emits that vmcnt(0) today
// whenever a copy is pending; the explicit wait keeps the order if a later edit makes the barrier a
// raw s_barrier.
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace ffc
