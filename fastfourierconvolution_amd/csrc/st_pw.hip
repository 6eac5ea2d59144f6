// SpectralTransform conv1 with the SE gate for large planes (gfx950):
//   t[b, o, p] = sum_c W[o, c] * gate[b, c] * x[b, c, p]        (spectral_transform.py:87-89)
// plus per-workgroup BatchNorm partials {n, mean, M2} of t for bn1 (:57,89).
//
// One workgroup = one sample x 256 pixels, all output channels.  The gated weight
// Wg[c][o] = W[o][c] * gate[b][c] of the sample is built once in LDS; each of the 4 waves streams
// 64 pixels of x (one global load per element, coalesced along the pixel row) through
// v_mfma_f32_32x32x2_f32 (exact fp32), K = Cin.  HBM traffic is x once + t once.
#include "ffc_internal.h"

namespace {

constexpr int PW_THREADS = 256;
constexpr int PW_PIX = 256;   // pixels per workgroup (64 per wave: two 32-column MFMA tiles)

struct PwArgs {
    const float* x;      // (B, Cin, HW)
    const float* gate;   // (B, Cin) or null
    const float* w;      // (M, Cin) conv1 weight
    float* t;            // (B, M, HW)
    float* slab;         // [B * nblk][M] float4 {n, mean, M2}, or null
    int Cin, M, HW, nblk, Mpad;
};

template <int MT>
__global__ __launch_bounds__(PW_THREADS) void pw_gate_kernel(PwArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Wg = smem;                               // [Cin][Mpad]
    float* scr = smem + a.Cin * a.Mpad;             // per-wave tile scratch / merge area
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hh = lane >> 5, col = lane & 31;
    const int b = blockIdx.x / a.nblk, blk = blockIdx.x - b * a.nblk;
    const int C = a.Cin, M = a.M;
    // 8 weight loads in flight per thread before their LDS stores (a load -> store loop would
    // serialise one L2 round trip per iteration)
    for (int i0 = 0; i0 < C * a.Mpad; i0 += 8 * PW_THREADS) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * PW_THREADS + tid;
            const int c = i / a.Mpad, o = i - c * a.Mpad;
            v[u] = 0.0f;
            if (i < C * a.Mpad && o < M)
                v[u] = a.w[(size_t)o * C + c] * (a.gate ? a.gate[(size_t)b * C + c] : 1.0f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * PW_THREADS + tid;
            if (i < C * a.Mpad) Wg[i] = v[u];
        }
    }
    __syncthreads();

    const int p0 = blk * PW_PIX + wave * 64;
    const float* xb = a.x + (size_t)b * C * a.HW;
    floatx16 acc[MT][2];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.0f;
    const int pa = p0 + col, pb = p0 + 32 + col;
    const bool va = pa < a.HW, vb = pb < a.HW;
    for (int c0 = 0; c0 < C; c0 += 16) {
        float xa[8], xbv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int c = c0 + 2 * u + hh;
            xa[u] = (c < C && va) ? xb[(size_t)c * a.HW + pa] : 0.0f;
            xbv[u] = (c < C && vb) ? xb[(size_t)c * a.HW + pb] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int c = c0 + 2 * u + hh;
            if (c0 + 2 * u < C) {
                const float* wr = Wg + min(c, C - 1) * a.Mpad + col;
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const float av = (c < C) ? wr[mt * 32] : 0.0f;
                    acc[mt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, xa[u], acc[mt][0], 0, 0, 0);
                    acc[mt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, xbv[u], acc[mt][1], 0, 0, 0);
                }
            }
        }
    }
    // store t
    float* tb = a.t + (size_t)b * M * a.HW;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (o < M) {
                if (va) tb[(size_t)o * a.HW + pa] = acc[mt][0][r];
                if (vb) tb[(size_t)o * a.HW + pb] = acc[mt][1][r];
            }
        }
    if (!a.slab) return;
    // BN partials: per 32-column tile (tile_row_stats), merged over the wave's two tiles, then
    // over the 4 waves in a fixed order -> one slab row per workgroup
    float st_n[MT], st_m[MT], st_q[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        st_n[mt] = st_m[mt] = st_q[mt] = 0.0f;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const int nv = max(0, min(32, a.HW - (p0 + 32 * nt)));
            if (nv == 0) continue;   // wave-uniform
            float mean, m2;
            ffc::tile_row_stats(acc[mt][nt], nv, scr + wave * ffc::TILE_SCRATCH, mean, m2);
            const float cn = (float)nv, tot = st_n[mt] + cn, d = mean - st_m[mt];
            st_m[mt] += d * (cn / tot);
            st_q[mt] += m2 + d * d * (st_n[mt] * cn / tot);
            st_n[mt] = tot;
        }
    }
    __syncthreads();
    float4* mg = reinterpret_cast<float4*>(scr);   // [wave][MT*32]
    if ((lane & 1) == 0) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
            mg[wave * MT * 32 + mt * 32 + (lane >> 1)] = make_float4(st_n[mt], st_m[mt], st_q[mt], 0.0f);
    }
    __syncthreads();
    for (int o = tid; o < M; o += PW_THREADS) {
        float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
        for (int wv = 0; wv < PW_THREADS / 64; ++wv) {
            const float4 e = mg[wv * MT * 32 + o];
            if (e.x > 0.0f) {
                const float tot = nn + e.x, d = e.y - mean;
                mean += d * (e.x / tot);
                m2 += e.z + d * d * (nn * e.x / tot);
                nn = tot;
            }
        }
        reinterpret_cast<float4*>(a.slab)[(size_t)blockIdx.x * M + o] = make_float4(nn, mean, m2, 0.0f);
    }
}

typedef void (*PwKernel)(PwArgs);

}  // namespace

extern "C" int ffc_pw_gate_blocks(int HW) { return HW > 0 ? (int)(((long long)HW + PW_PIX - 1) / PW_PIX) : 0; }

extern "C" size_t ffc_pw_gate_lds_bytes(int Cin, int M) {
    if (Cin <= 0 || M <= 0 || M > 128) return 0;
    const size_t Mpad = (size_t)(M + 31) / 32 * 32;
    const size_t bytes = 4 * ((size_t)Cin * Mpad + (PW_THREADS / 64) * ffc::TILE_SCRATCH);
    return bytes <= 160 * 1024 ? bytes : 0;
}

extern "C" int ffc_pw_gate_conv(const float* x, const float* gate, const float* w, int B, int Cin, int M, int HW,
                                float* t, float* slab, void* stream) {
    FFC_CHECK_ARG(x && w && t && B > 0 && HW > 0, "ffc_pw_gate_conv: bad args");
    const size_t lds = ffc_pw_gate_lds_bytes(Cin, M);
    FFC_CHECK_ARG(lds > 0, "ffc_pw_gate_conv: unsupported (Cin, M): M <= 128 and Cin*ceil32(M) floats in LDS");
    PwArgs a;
    a.x = x;
    a.gate = gate;
    a.w = w;
    a.t = t;
    a.slab = slab;
    a.Cin = Cin;
    a.M = M;
    a.HW = HW;
    a.nblk = ffc_pw_gate_blocks(HW);
    a.Mpad = (M + 31) / 32 * 32;
    PwKernel k = a.Mpad <= 32 ? pw_gate_kernel<1> : a.Mpad <= 64 ? pw_gate_kernel<2> : pw_gate_kernel<4>;
    if (lds > 64 * 1024) {
        static bool raised[3] = {false, false, false};
        const int i = a.Mpad <= 32 ? 0 : a.Mpad <= 64 ? 1 : 2;
        if (!raised[i]) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    160 * 1024) != hipSuccess) {
                ffc::set_error("ffc_pw_gate_conv: hipFuncSetAttribute failed");
                return FFC_E_LAUNCH;
            }
            raised[i] = true;
        }
    }
    hipLaunchKernelGGL(k, dim3((unsigned)(B * a.nblk)), dim3(PW_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_pw_gate_conv");
}
