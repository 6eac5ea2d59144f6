// Dense GEMM + bias + activation for gfx950 (v_mfma_f32_32x32x2_f32, exact fp32):
//   out[b][n] = act(sum_k A[b][k] * Wt[k][n] + bias[n])
// Used where a layer is a plain matrix product:
//   - ConvTranspose2d(k, s=1, p=0) on a 1x1 input (the FFC-DCGAN generator's first layer,
//     models/ffc_generator.py:24; ffc_transpose.py:79-86): n = (m, ky, kx), so the (B, M*k*k)
//     result IS the (B, M, k, k) output; its l and g branches go to two outputs of one launch.
//   - the fgan128 generator's nn.Linear(z, 16*1024) (fgan128_complete.py:453-455).
// Workgroup tile: 64 rows (b) x 64 columns (n), A staged in LDS; each of the 4 waves owns 32 x 32.
#include "ffc_internal.h"

#include <cstdlib>

namespace {

constexpr int DN_THREADS = 256;
constexpr int DN_BM = 64, DN_BN = 64;   // 4 waves, each 32 x 32
constexpr int DN_KMAX = 256;            // A tile (64 x K) staged in LDS, rows padded to K+1

struct DenseArgs {
    const float* A;      // (B, K)
    const float* Wt;     // (K, N) row-major
    const float* bias;   // (N) or null
    float* out0;         // columns [0, N0): (B, N0)
    float* out1;         // columns [N0, N): (B, N - N0), or null when N0 == N
    int B, K, N, N0;
    int act;
    float act_param;
};

// VEC: the W tile (K x 64) and the A tile staged with 16-byte loads (K % 4 == 0, N % 4 == 0, aligned
// rows): 16 vector loads per thread instead of 96 scalar ones; W is read back from LDS with odd k
// rows rotated by 32 columns (the two lane halves read rows 2u and 2u+1: different banks)
template <int KH, bool VEC>
__global__ __launch_bounds__(DN_THREADS) void dense_kernel(DenseArgs a) {
    extern __shared__ float As[];   // [64][K+1]  (VEC: then Ws [2 KH][64])
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hh = lane >> 5, col = lane & 31;
    const int ntn = (a.N + DN_BN - 1) / DN_BN;
    const int tm = blockIdx.x / ntn, tn = blockIdx.x - tm * ntn;
    const int b0 = tm * DN_BM;
    const int KS = 2 * KH + 1;   // rows zero-padded to 2 KH: the MFMA loop reads without bounds checks
    const auto rA = ffc::buf_rsrc(a.A, (unsigned long long)a.B * a.K * 4);
    const auto rW = ffc::buf_rsrc(a.Wt, (unsigned long long)a.K * a.N * 4);
    const int wr = wave >> 1, wc = wave & 1;
    const int n = tn * DN_BN + wc * 32 + col;
    const bool nv = n < a.N;
    // every global load of the workgroup in flight at once -- the lane's whole W column (k = 2u + hh,
    // K <= 2 KH) and its share of the 64 x K A tile -- so the launch pays one memory latency
    // (bounds-checked buffer loads: out-of-range elements read 0, no branch per load)
    float wa[VEC ? 1 : KH];
    float* Ws = As + DN_BM * KS;
    if constexpr (VEC) {
        // W rows k, 64 columns from tn * 64: 16 groups of 4 per row; out-of-range groups read 0
        constexpr int NG = 2 * KH * 16 / DN_THREADS;
#pragma unroll
        for (int j = 0; j < NG; ++j) {
            const int i = j * DN_THREADS + tid, k = i >> 4, c4 = i & 15;
            const int nn = tn * DN_BN + 4 * c4;
            const bool ok = k < a.K && nn < a.N;
            const floatx4 w4 = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                rW, ok ? (int)(((size_t)k * a.N + nn) * 4) : (int)ffc::OOB, 0, 0));
            *reinterpret_cast<floatx4*>(Ws + k * 64 + ((4 * c4 + 32 * (k & 1)) & 63)) = w4;
        }
    } else {
#pragma unroll
        for (int u = 0; u < KH; ++u) {
            const int k = 2 * u + hh;
            const bool ok = k < a.K && nv;
            wa[u] = ffc::buf_ld(rW, ok ? (unsigned)(((size_t)k * a.N + n) * 4) : ffc::OOB);
        }
    }
    // the 64 x K A tile: wave w stages rows 16w .. 16w+15, lane l columns l, l+64, .. (< 2 KH), zeros
    // past K -- row / column come from the lane and loop indices (no per-element division by K)
    constexpr int NC = 2 * KH / 64;                   // column groups of 64 (K <= 2 KH)
    constexpr int NA = (DN_BM / 4) * NC;               // A elements per thread
    if constexpr (VEC) {
        // the 64 x 2KH A tile as 16-byte groups (rows b0 .., K % 4 == 0): 2KH / 4 groups per row
        constexpr int GR = 2 * KH / 4, NGA = DN_BM * GR / DN_THREADS;
#pragma unroll
        for (int j = 0; j < NGA; ++j) {
            const int i = j * DN_THREADS + tid, r = i / GR, k4 = i - r * GR;
            const bool ok = 4 * k4 < a.K && b0 + r < a.B;
            const floatx4 v4 = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                rA, ok ? (int)(((size_t)(b0 + r) * a.K + 4 * k4) * 4) : (int)ffc::OOB, 0, 0));
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (4 * k4 + e < KS) As[r * KS + 4 * k4 + e] = v4[e];
        }
    }
    float v[VEC ? 1 : NA];
    if constexpr (!VEC) {
#pragma unroll
    for (int rr = 0; rr < DN_BM / 4; ++rr)
#pragma unroll
        for (int cg = 0; cg < NC; ++cg) {
            const int r = wave * (DN_BM / 4) + rr, k = cg * 64 + lane;
            const bool ok = k < a.K && b0 + r < a.B;
            v[rr * NC + cg] = ffc::buf_ld(rA, ok ? (unsigned)(((size_t)(b0 + r) * a.K + k) * 4) : ffc::OOB);
        }
#pragma unroll
    for (int rr = 0; rr < DN_BM / 4; ++rr)
#pragma unroll
        for (int cg = 0; cg < NC; ++cg) {
            const int r = wave * (DN_BM / 4) + rr, k = cg * 64 + lane;
            if (k < KS) As[r * KS + k] = v[rr * NC + cg];   // out-of-range loads read 0: the row tails
        }
    }
    __syncthreads();
    const float* ar = As + (wr * 32 + col) * KS;   // this lane's A row
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    const int ku = (a.K + 1) >> 1;   // k-steps that hold data (k >= K: zero A and zero W)
    // in groups of 4 k-steps, a group wholly past K skipped (wave-uniform branch): K = 100 runs 52
    // of the 64 MFMAs
#pragma unroll
    for (int u0 = 0; u0 < KH; u0 += 4) {
        if (u0 < ku) {
#pragma unroll
            for (int u = u0; u < u0 + 4; ++u) {
                float wv;
                if constexpr (VEC) wv = Ws[(2 * u + hh) * 64 + ((wc * 32 + col + 32 * hh) & 63)];
                else wv = wa[u];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * u + hh], wv, acc, 0, 0, 0);
            }
        }
    }
    if (!nv) return;
    const float bv = a.bias ? a.bias[n] : 0.0f;
    // argument fields read before the stores (after a store the compiler reloads them)
    float* dst;
    int ld;
    if (n < a.N0) {
        dst = a.out0 + n;
        ld = a.N0;
    } else {
        dst = a.out1 + (n - a.N0);
        ld = a.N - a.N0;
    }
    const int Bn = a.B, act = a.act;
    const float ap = a.act_param;
    auto store = [&](auto actf) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int b = b0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (b < Bn) dst[(size_t)b * ld] = actf(acc[r] + bv);
        }
    };
    switch (act) {   // one branch per launch, not per element
        case FFC_ACT_IDENTITY: store([](float v) { return v; }); break;
        case FFC_ACT_RELU: store([](float v) { return fmaxf(v, 0.0f); }); break;
        case FFC_ACT_LEAKY_RELU: store([ap](float v) { return v > 0.0f ? v : v * ap; }); break;
        default: store([act, ap](float v) { return ffc::apply_act(v, act, ap); }); break;
    }
}

}  // namespace

extern "C" int ffc_dense_forward(const float* A, const float* Wt, const float* bias, int B, int K, int N, int N0,
                                 float* out0, float* out1, int act, float act_param, void* stream) {
    FFC_CHECK_ARG(A && Wt && out0 && B > 0 && K > 0 && N > 0, "ffc_dense_forward: bad args");
    FFC_CHECK_ARG(N0 > 0 && N0 <= N && (N0 == N || out1 != nullptr), "ffc_dense_forward: output split");
    FFC_CHECK_ARG(K <= DN_KMAX, "ffc_dense_forward: K > 256");
    DenseArgs a{A, Wt, bias, out0, out1, B, K, N, N0, act, act_param};
    const int grid = ((B + DN_BM - 1) / DN_BM) * ((N + DN_BN - 1) / DN_BN);
    const int KH = K <= 128 ? 64 : 128;
    static const bool vec_on = [] {   // FFC_DENSE_VEC=0: the scalar-load staging (A/B)
        const char* e = std::getenv("FFC_DENSE_VEC");
        return !(e && e[0] == '0');
    }();
    const bool vec = vec_on && K % 4 == 0 && N % 4 == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(Wt) & 15) == 0;
    const size_t lds = sizeof(float) * (DN_BM * (2 * KH + 1) + (vec ? 2 * KH * 64 : 0));
    typedef void (*DenseKernel)(DenseArgs);
    static const DenseKernel kernels[2][2] = {{dense_kernel<64, false>, dense_kernel<64, true>},
                                              {dense_kernel<128, false>, dense_kernel<128, true>}};
    const DenseKernel k = kernels[KH == 128][vec];
    if (lds > 64 * 1024) {
        static bool raised[2][2] = {};
        if (!raised[KH == 128][vec]) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    160 * 1024) != hipSuccess) {
                ffc::set_error("ffc_dense_forward: hipFuncSetAttribute failed");
                return FFC_E_LAUNCH;
            }
            raised[KH == 128][vec] = true;
        }
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(DN_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_dense_forward");
}
