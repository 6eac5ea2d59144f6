// Training path (BASELINE config 3: FFC-DCGAN generator + discriminator fwd+bwd) on gfx950.
//
// The inference forward fuses whole SpectralTransforms into a few launches and keeps nothing.
// With autograd the path is split at the reference's own op boundaries (fourier_unity.py:32-56,
// spectral_transform.py:77-110, ffc.py:84-99, ffc_transpose.py:91-110, ffc_bn_act.py:70-83),
// each op a custom autograd function over the kernels below plus the inference conv GEMMs,
// which also compute every data gradient (the adjoint of a conv is a transposed conv with the
// same weight tensor and vice versa, so ffc_conv_forward / ffc_convp_forward run them):
//
//   ffc_conv_wgrad        weight gradients of conv / convT / 1x1 / Linear on f32 MFMA
//                         (v_mfma_f32_32x32x2_f32), split-K over samples, deterministic
//   ffc_rfft2_planes      rfftn(norm="ortho") per plane into the interleaved Re/Im channel
//                         planes of fourier_unity.py:40-42 (interior bins x scale: with 2 it is
//                         the adjoint of irfftn)
//   ffc_irfft2_planes     irfftn(s=(H,W), norm="ortho") from interleaved planes (+ addend);
//                         interior bins x scale (0.5 gives the adjoint of rfftn)
//   ffc_channel_moments   {n, sum x, sum x^2} per channel in fp64 (BatchNorm2d batch stats)
//   ffc_bn_bwd_*          BatchNorm2d (+ following activation) backward, fp64 reductions
//   ffc_act_bwd           activation backward from the activation output
//   ffc_se_bwd            SELayer backward, one workgroup per sample
//   ffc_pool2 / ffc_up2   2x2 average pool / nearest x2 upsample (and each other's adjoint)
#include <algorithm>

#include "ffc_internal.h"

#include <cstdlib>

namespace {

__device__ __forceinline__ float act_grad_from_out(float y, float x_or_y, int act, float p) {
    // derivative of the activation expressed through its output y (GELU: through its input)
    switch (act) {
        case FFC_ACT_RELU: return y > 0.0f ? 1.0f : 0.0f;
        case FFC_ACT_LEAKY_RELU: return y > 0.0f ? 1.0f : p;
        case FFC_ACT_TANH: return 1.0f - y * y;
        case FFC_ACT_SIGMOID: return y * (1.0f - y);
        case FFC_ACT_GELU: {
            const float x = x_or_y;
            const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
            const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
            return cdf + x * pdf;
        }
        default: return 1.0f;
    }
}

// ------------------------------------------------------------------ activation backward
__global__ void act_bwd_kernel(const float* __restrict__ t, const float* __restrict__ dy, float* __restrict__ dx,
                               long long n, int act, float p) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float v = t[i];
        float y = v;
        if (act == FFC_ACT_GELU) y = 0.0f;
        dx[i] = dy[i] * act_grad_from_out(y, v, act, p);
    }
}

// ------------------------------------------------------------------ channel moments (fp64)
// grid (C, S): workgroup (c, s) sums its share of the B*HW elements of channel c
__global__ void moments_partial_kernel(const float* __restrict__ x, int B, int C, int HW, int S,
                                       double* __restrict__ ws) {
    const int c = blockIdx.x, s = blockIdx.y;
    const long long per = (long long)B * HW;
    const long long lo = per * s / S, hi = per * (s + 1) / S;
    double s1 = 0.0, s2 = 0.0;
    for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        const long long b = i / HW, q = i - b * HW;
        const double v = x[((size_t)b * C + c) * HW + q];
        s1 += v;
        s2 += v * v;
    }
    __shared__ double r1[256], r2[256];
    r1[threadIdx.x] = s1;
    r2[threadIdx.x] = s2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            r1[threadIdx.x] += r1[threadIdx.x + o];
            r2[threadIdx.x] += r2[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        ws[((size_t)s * C + c) * 2] = r1[0];
        ws[((size_t)s * C + c) * 2 + 1] = r2[0];
    }
}

__global__ void moments_final_kernel(const double* __restrict__ ws, int S, int C, double count, double* moments) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double s1 = 0.0, s2 = 0.0;
    for (int s = 0; s < S; ++s) {
        s1 += ws[((size_t)s * C + c) * 2];
        s2 += ws[((size_t)s * C + c) * 2 + 1];
    }
    moments[3 * c] = count;
    moments[3 * c + 1] = s1;
    moments[3 * c + 2] = s2;
}

// ------------------------------------------------------------------ BatchNorm2d (+act) backward
// g = dy * act'(act(x*scale + shift)); partial sums of g and g*x per channel
__global__ void bn_bwd_partial_kernel(const float* __restrict__ x, const float* __restrict__ dy, int B, int C, int HW,
                                      int S, const float* __restrict__ scale, const float* __restrict__ shift, int act,
                                      float p, double* __restrict__ ws) {
    const int c = blockIdx.x, s = blockIdx.y;
    const long long per = (long long)B * HW;
    const long long lo = per * s / S, hi = per * (s + 1) / S;
    const float sc = scale[c], sh = shift[c];
    double s1 = 0.0, s2 = 0.0;
    for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        const long long b = i / HW, q = i - b * HW;
        const size_t off = ((size_t)b * C + c) * HW + q;
        const float xv = x[off];
        const float z = fmaf(xv, sc, sh);
        const float g = dy[off] * act_grad_from_out(ffc::apply_act(z, act, p), z, act, p);
        s1 += g;
        s2 += (double)g * xv;
    }
    __shared__ double r1[256], r2[256];
    r1[threadIdx.x] = s1;
    r2[threadIdx.x] = s2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            r1[threadIdx.x] += r1[threadIdx.x + o];
            r2[threadIdx.x] += r2[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        ws[((size_t)s * C + c) * 2] = r1[0];
        ws[((size_t)s * C + c) * 2 + 1] = r2[0];
    }
}

// per channel: mean/invstd exactly as the forward finalize (bn_se_kernels.hip finalize_channel),
// then dx = k0*g + k1*x + k2, dgamma = sum g*xhat, dbeta = sum g
__global__ void bn_bwd_coeff_kernel(const double* __restrict__ ws, int S, int C, const double* __restrict__ moments,
                                    const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
                                    const float* __restrict__ gamma, float* __restrict__ coef,
                                    float* __restrict__ dgamma, float* __restrict__ dbeta) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double sg = 0.0, sgx = 0.0;
    for (int s = 0; s < S; ++s) {
        sg += ws[((size_t)s * C + c) * 2];
        sgx += ws[((size_t)s * C + c) * 2 + 1];
    }
    float mean, var;
    double n = 0.0;
    if (moments) {
        n = moments[3 * c];
        const double mu = moments[3 * c + 1] / n;
        double v = moments[3 * c + 2] / n - mu * mu;
        if (v < 0.0) v = 0.0;
        mean = (float)mu;
        var = (float)v;
    } else {
        mean = rmean[c];
        var = rvar[c];
    }
    const float inv = 1.0f / sqrtf(var + eps);
    const float gm = gamma ? gamma[c] : 1.0f;
    const double sgxh = (sgx - (double)mean * sg) * (double)inv;   // sum g * xhat
    if (dgamma) dgamma[c] = (float)sgxh;
    if (dbeta) dbeta[c] = (float)sg;
    const float k0 = gm * inv;
    float k1 = 0.0f, k2 = 0.0f;
    if (moments) {
        const double a = sgxh / n * (double)inv;   // coefficient of (x - mean) * inv
        k1 = (float)(-(double)k0 * a);
        k2 = (float)((double)k0 * (a * (double)mean - sg / n));
    }
    coef[3 * c] = k0;
    coef[3 * c + 1] = k1;
    coef[3 * c + 2] = k2;
}

__global__ void bn_bwd_apply_kernel(const float* __restrict__ x, const float* __restrict__ dy, int C, int HW,
                                    long long total, const float* __restrict__ scale, const float* __restrict__ shift,
                                    int act, float p, const float* __restrict__ coef, float* __restrict__ dx) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)((i / HW) % C);
        const float xv = x[i];
        const float z = fmaf(xv, scale[c], shift[c]);
        const float g = dy[i] * act_grad_from_out(ffc::apply_act(z, act, p), z, act, p);
        dx[i] = fmaf(coef[3 * c], g, fmaf(coef[3 * c + 1], xv, coef[3 * c + 2]));
    }
}

// ------------------------------------------------------------------ weight gradient (MFMA)
// G[m][n*T + t] = sum_b sum_q U[b][m][q] * V[b][n][qy*s - p + kh*d][qx*s - p + kw*d]
// (zero outside V), t = kh*k + kw, q = qy*PW + qx.  K = (b, q) flattened, chunks staged in LDS;
// 128x128 or 64x64 tile per workgroup, 4 waves of v_mfma_f32_32x32x2_f32 tiles.
// grid (tiles_n, tiles_m, S): split z reduces samples [B*z/S, B*(z+1)/S) into ws[z] (or into
// G directly when S == 1).
struct WgradArgs {
    const float* U;
    const float* V;
    float* out;   // ws [S][Mu][NT] or G
    int B, Mu, PH, PW, Nv, VH, VW, k, s, p, d, S;
};

// BT x BT tile (64 or 128), each wave a (BT/2) x (BT/2) quadrant of TT x TT MFMA tiles; K in
// BK-deep chunks (64 for the small tile: its chunk carries only 8 MFMAs per wave, so the loads of
// four 16-deep chunks are issued together to pay the global-load latency once; 32 for the large
// tile: 64 MFMAs per wave between barriers)
template <int BT, int BK, bool SPLIT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_kernel(WgradArgs a) {
    constexpr int WG_BK = BK;
    constexpr int WG_LD = BK + 1;
    constexpr int RS = 256 / BK;       // row stride between a thread's staged rows
    constexpr int R = BT / RS;         // rows of A / columns of B each thread stages per chunk
    constexpr int TT = BT / 64;        // 32x32 MFMA tiles per wave per dimension
    __shared__ float As[BT * WG_LD];
    __shared__ float Bs[BT * WG_LD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = a.k * a.k, NT = a.Nv * T, P = a.PH * a.PW;
    const int m0 = blockIdx.y * BT, n0 = blockIdx.x * BT, z = blockIdx.z;
    // split z reduces k = (sample, pixel) in [K0, K1): an even share of the flattened K
    const long long Ktot = (long long)a.B * P;
    const long long K0 = Ktot * z / a.S, K1 = Ktot * (z + 1) / a.S;
    const size_t VP = (size_t)a.VH * a.VW;
    // this thread's k column and its R rows (A) / R columns (B) of every chunk
    const int kc = tid % BK, rbase = tid / BK;
    int vn[R], vky[R], vkx[R];
    bool vok[R], aok[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int col = n0 + rbase + RS * r;
        vok[r] = col < NT;
        const int n = vok[r] ? col / T : 0, t = vok[r] ? col - n * T : 0;
        vn[r] = n;
        vky[r] = (t / a.k) * a.d - a.p;
        vkx[r] = (t % a.k) * a.d - a.p;
        aok[r] = m0 + rbase + RS * r < a.Mu;
    }
    floatx16 acc[TT][TT];
#pragma unroll
    for (int i = 0; i < TT; ++i)
#pragma unroll
        for (int j = 0; j < TT; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
    const int wm = (wave >> 1) * (BT / 2), wn = (wave & 1) * (BT / 2);
    const int h = lane >> 5, cl = lane & 31;
    float av[R], bv[R];
    auto load_chunk = [&](long long kk0) {
        const long long kk = kk0 + kc;
        if (kk < K1) {
            const int b = (int)(kk / P), q = (int)(kk - (long long)b * P);
            const int qy = q / a.PW, qx = q - qy * a.PW;
            const float* Ub = a.U + ((size_t)b * a.Mu) * P + q;
            const float* Vb = a.V + (size_t)b * a.Nv * VP;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                av[r] = aok[r] ? Ub[(size_t)(m0 + rbase + RS * r) * P] : 0.0f;
                const int iy = qy * a.s + vky[r], ix = qx * a.s + vkx[r];
                bv[r] = (vok[r] && iy >= 0 && iy < a.VH && ix >= 0 && ix < a.VW)
                            ? Vb[(size_t)vn[r] * VP + (size_t)iy * a.VW + ix] : 0.0f;
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) av[r] = bv[r] = 0.0f;
        }
    };
    if (K0 < K1) load_chunk(K0);
    for (long long kk0 = K0; kk0 < K1; kk0 += WG_BK) {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            As[(rbase + RS * r) * WG_LD + kc] = av[r];
            Bs[(rbase + RS * r) * WG_LD + kc] = bv[r];
        }
        __syncthreads();
        if (kk0 + WG_BK < K1) load_chunk(kk0 + WG_BK);   // next chunk's loads overlap this chunk's MFMAs
        if constexpr (SPLIT) {
            // fp32-accurate split-bf16 MFMA (ffc_internal.h split3): per 16-deep k-step, element j
            // of lane half h is k = 2j + h for both operands (k-steps not unrolled: register budget)
#pragma unroll 1
            for (int q = 0; q < WG_BK / 16; ++q) {
                Split3 ys[TT];
#pragma unroll
                for (int j = 0; j < TT; ++j) {
                    float yv[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) yv[e] = Bs[(wn + 32 * j + cl) * WG_LD + 16 * q + 2 * e + h];
                    ys[j] = split3(yv);
                }
#pragma unroll
                for (int i = 0; i < TT; ++i) {
                    float xv[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) xv[e] = As[(wm + 32 * i + cl) * WG_LD + 16 * q + 2 * e + h];
                    const Split3 xs = split3(xv);
#pragma unroll
                    for (int j = 0; j < TT; ++j) acc[i][j] = mfma_split3(xs, ys[j], acc[i][j]);
                }
            }
            continue;
        }
#pragma unroll
        for (int st = 0; st < WG_BK / 2; ++st) {
            float x[TT], y[TT];
#pragma unroll
            for (int i = 0; i < TT; ++i) {
                x[i] = As[(wm + 32 * i + cl) * WG_LD + 2 * st + h];
                y[i] = Bs[(wn + 32 * i + cl) * WG_LD + 2 * st + h];
            }
#pragma unroll
            for (int i = 0; i < TT; ++i)
#pragma unroll
                for (int j = 0; j < TT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[i], y[j], acc[i][j], 0, 0, 0);
        }
    }
    float* out = a.out + (size_t)z * a.Mu * NT;
#pragma unroll
    for (int j = 0; j < TT; ++j) {
        const int col = n0 + wn + 32 * j + cl;
        if (col >= NT) continue;
#pragma unroll
        for (int i = 0; i < TT; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < a.Mu) out[(size_t)m * NT + col] = acc[i][j][r];
            }
    }
}

// Split-once variant (default): each staged element is split into its three exact bf16 pieces
// once, when the workgroup writes the chunk to LDS (three bf16 planes per operand), instead of per
// use by every wave that reads it; the MFMA loop then reads each operand fragment as three
// ds_read_b128 (8 consecutive k per lane: the lane-half h of a 32x32x16 bf16 fragment holds
// k = 8h .. 8h + 7, the same mapping for both operands).  Staging: a thread owns 8 consecutive k of
// one row per group; when P % 8 == 0 the group lies in one sample, so U comes in as two float4 and
// the V gather walks its 8 pixels incrementally; the K split is then cut on 8-k boundaries.
// Row stride 40 bf16 (80 B = 20 dwords): the 16 rows of a ds_read_b128 group hit distinct banks.
template <int BM, int BN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgradq_kernel(WgradArgs a) {
    constexpr int BK = 32, LDR = 40;
    constexpr int GA = BM * BK / 8 / 256, GB = BN * BK / 8 / 256;   // 8-k groups per thread
    constexpr int TM = BM / 64, TN = BN / 64;                       // 32x32 tiles per wave per dimension
    static_assert(GA >= 1 && GB >= 1, "tile too small for 256 staging threads");
    __shared__ __attribute__((aligned(16))) unsigned short As[3][BM * LDR];
    __shared__ __attribute__((aligned(16))) unsigned short Bs[3][BN * LDR];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = a.k * a.k, NT = a.Nv * T, P = a.PH * a.PW;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN, z = blockIdx.z;
    const bool vec = (P & 7) == 0;
    const long long Ktot = (long long)a.B * P;
    long long K0, K1;
    if (vec) {
        const long long K8 = Ktot >> 3;
        K0 = (K8 * z / a.S) << 3;
        K1 = (K8 * (z + 1) / a.S) << 3;
    } else {
        K0 = Ktot * z / a.S;
        K1 = Ktot * (z + 1) / a.S;
    }
    const size_t VP = (size_t)a.VH * a.VW;
    const int kq = tid & 3;          // this thread's 8-k group within a chunk: k = 8 kq .. 8 kq + 7
    const int rb = tid >> 2;         // row of its first group; further groups 64 rows apart
    bool aok[GA], vok[GB];
    int vn[GB], vky[GB], vkx[GB];
#pragma unroll
    for (int g = 0; g < GA; ++g) aok[g] = m0 + rb + 64 * g < a.Mu;
#pragma unroll
    for (int g = 0; g < GB; ++g) {
        const int col = n0 + rb + 64 * g;
        vok[g] = col < NT;
        const int n = vok[g] ? col / T : 0, t = vok[g] ? col - n * T : 0;
        vn[g] = n;
        vky[g] = (t / a.k) * a.d - a.p;
        vkx[g] = (t % a.k) * a.d - a.p;
    }
    float av[GA][8], bv[GB][8];
    auto load_chunk = [&](long long kk0) {
        const long long kb = kk0 + 8 * kq;
        if (vec) {
            if (kb < K1) {
                const int b = (int)(kb / P), q0 = (int)(kb - (long long)b * P);
#pragma unroll
                for (int g = 0; g < GA; ++g) {
                    if (aok[g]) {
                        const float4* u = reinterpret_cast<const float4*>(
                            a.U + ((size_t)b * a.Mu + m0 + rb + 64 * g) * P + q0);
                        const float4 u0 = u[0], u1 = u[1];
                        av[g][0] = u0.x; av[g][1] = u0.y; av[g][2] = u0.z; av[g][3] = u0.w;
                        av[g][4] = u1.x; av[g][5] = u1.y; av[g][6] = u1.z; av[g][7] = u1.w;
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) av[g][e] = 0.0f;
                    }
                }
                const int qy0 = q0 / a.PW, qx0 = q0 - qy0 * a.PW;
                const float* Vb = a.V + (size_t)b * a.Nv * VP;
#pragma unroll
                for (int g = 0; g < GB; ++g) {
                    int qy = qy0, qx = qx0;
                    const float* Vn = Vb + (size_t)vn[g] * VP;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int iy = qy * a.s + vky[g], ix = qx * a.s + vkx[g];
                        bv[g][e] = (vok[g] && iy >= 0 && iy < a.VH && ix >= 0 && ix < a.VW)
                                       ? Vn[(size_t)iy * a.VW + ix] : 0.0f;
                        if (++qx == a.PW) { qx = 0; ++qy; }
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
#pragma unroll
                    for (int g = 0; g < GA; ++g) av[g][e] = 0.0f;
#pragma unroll
                    for (int g = 0; g < GB; ++g) bv[g][e] = 0.0f;
                }
            }
            return;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const long long kk = kb + e;
            const bool ok = kk < K1;
            const int b = ok ? (int)(kk / P) : 0, q = ok ? (int)(kk - (long long)b * P) : 0;
            const int qy = q / a.PW, qx = q - qy * a.PW;
#pragma unroll
            for (int g = 0; g < GA; ++g)
                av[g][e] = (ok && aok[g]) ? a.U[((size_t)b * a.Mu + m0 + rb + 64 * g) * P + q] : 0.0f;
            const float* Vb = a.V + (size_t)b * a.Nv * VP;
#pragma unroll
            for (int g = 0; g < GB; ++g) {
                const int iy = qy * a.s + vky[g], ix = qx * a.s + vkx[g];
                bv[g][e] = (ok && vok[g] && iy >= 0 && iy < a.VH && ix >= 0 && ix < a.VW)
                               ? Vb[(size_t)vn[g] * VP + (size_t)iy * a.VW + ix] : 0.0f;
            }
        }
    };
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
    const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
    const int h = lane >> 5, cl = lane & 31;
    if (K0 < K1) load_chunk(K0);
    for (long long kk0 = K0; kk0 < K1; kk0 += BK) {
        __syncthreads();
#pragma unroll
        for (int g = 0; g < GA; ++g) {
            const Split3 sp = split3(av[g]);
            const int o = (rb + 64 * g) * LDR + 8 * kq;
            *reinterpret_cast<bf16x8*>(&As[0][o]) = sp.hi;
            *reinterpret_cast<bf16x8*>(&As[1][o]) = sp.mid;
            *reinterpret_cast<bf16x8*>(&As[2][o]) = sp.lo;
        }
#pragma unroll
        for (int g = 0; g < GB; ++g) {
            const Split3 sp = split3(bv[g]);
            const int o = (rb + 64 * g) * LDR + 8 * kq;
            *reinterpret_cast<bf16x8*>(&Bs[0][o]) = sp.hi;
            *reinterpret_cast<bf16x8*>(&Bs[1][o]) = sp.mid;
            *reinterpret_cast<bf16x8*>(&Bs[2][o]) = sp.lo;
        }
        __syncthreads();
        if (kk0 + BK < K1) load_chunk(kk0 + BK);   // next chunk's loads overlap this chunk's MFMAs
#pragma unroll
        for (int q = 0; q < BK / 16; ++q) {
            Split3 ys[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int o = (wn + 32 * j + cl) * LDR + 16 * q + 8 * h;
                ys[j].hi = *reinterpret_cast<const bf16x8*>(&Bs[0][o]);
                ys[j].mid = *reinterpret_cast<const bf16x8*>(&Bs[1][o]);
                ys[j].lo = *reinterpret_cast<const bf16x8*>(&Bs[2][o]);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int o = (wm + 32 * i + cl) * LDR + 16 * q + 8 * h;
                Split3 xs;
                xs.hi = *reinterpret_cast<const bf16x8*>(&As[0][o]);
                xs.mid = *reinterpret_cast<const bf16x8*>(&As[1][o]);
                xs.lo = *reinterpret_cast<const bf16x8*>(&As[2][o]);
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma_split3(xs, ys[j], acc[i][j]);
            }
        }
    }
    float* out = a.out + (size_t)z * a.Mu * NT;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn + 32 * j + cl;
        if (col >= NT) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < a.Mu) out[(size_t)m * NT + col] = acc[i][j][r];
            }
    }
}

int wgrad_tile(int Mu, int NT) { return (Mu >= 128 && NT >= 128) ? 128 : 64; }

// few weights, many splits: 16 weights x 16 split groups per workgroup, fixed-order LDS combine
__global__ __launch_bounds__(256) void split_sum_grouped_kernel(const float* __restrict__ ws, int S, long long n,
                                                                float* __restrict__ out, int accumulate) {
    __shared__ float part[16][17];
    const int e = threadIdx.x & 15, g = threadIdx.x >> 4;
    const long long i = (long long)blockIdx.x * 16 + e;
    float v = 0.0f;
    if (i < n)
        for (int s = g; s < S; s += 16) v += ws[(size_t)s * n + i];
    part[g][e] = v;
    __syncthreads();
    if (g == 0 && i < n) {
        float t = 0.0f;
#pragma unroll
        for (int q = 0; q < 16; ++q) t += part[q][e];
        out[i] = accumulate ? out[i] + t : t;
    }
}

__global__ void split_sum_kernel(const float* __restrict__ ws, int S, long long n, float* __restrict__ out,
                                 int accumulate) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        float v = 0.0f;
        for (int s = 0; s < S; ++s) v += ws[(size_t)s * n + i];
        out[i] = accumulate ? out[i] + v : v;
    }
}

// ------------------------------------------------------------------ planar 2-D real DFTs
// One workgroup handles NPW planes.  Twiddles tw[j] = exp(-2 pi i j / N) in LDS (fp64 sincospi
// rounded once).  Direct DFT sums: plane sizes on the training path are 4..64 per side.
constexpr int DFT_MAXN = 64;

__device__ __forceinline__ void make_twiddles(float2* tw, int N, int tid, int nt) {
    for (int j = tid; j < N; j += nt) {
        double sn, cs;
        sincospi(2.0 * j / N, &sn, &cs);
        tw[j] = make_float2((float)cs, (float)-sn);
    }
}

__device__ __forceinline__ float interior_weight(int kw, int W) {
    return (kw == 0 || 2 * kw == W) ? 0.0f : 1.0f;   // 1 where the bin has a Hermitian mirror
}

// x planes (P, H, W) -> Z: Re of plane p at Z + 2p*H*W', Im at Z + (2p+1)*H*W'
__global__ __launch_bounds__(256) void rfft2_kernel(const float* __restrict__ x, int P, int H, int W, int NPW,
                                                    float iscale, float* __restrict__ Z) {
    extern __shared__ float smem[];
    const int Wp = W / 2 + 1, HWp = H * Wp, HW = H * W;
    float2* twW = reinterpret_cast<float2*>(smem);
    float2* twH = twW + DFT_MAXN;
    float* xs = reinterpret_cast<float*>(twH + DFT_MAXN);          // NPW * HW
    float2* R = reinterpret_cast<float2*>(xs + NPW * HW);          // NPW * HWp
    const int tid = threadIdx.x;
    const int p0 = blockIdx.x * NPW;
    const int np = min(NPW, P - p0);
    make_twiddles(twW, W, tid, 256);
    make_twiddles(twH, H, tid, 256);
    for (int i = tid; i < np * HW; i += 256) xs[i] = x[(size_t)p0 * HW + i];
    __syncthreads();
    // rows: R[h][kw] = sum_w x[h][w] e^{-2 pi i kw w / W}
    for (int i = tid; i < np * HWp; i += 256) {
        const int pl = i / HWp, r = i - pl * HWp, hh = r / Wp, kw = r - hh * Wp;
        const float* row = xs + pl * HW + hh * W;
        float re = 0.0f, im = 0.0f;
        int j = 0;
        for (int w = 0; w < W; ++w) {
            const float2 t = twW[j];
            re = fmaf(row[w], t.x, re);
            im = fmaf(row[w], t.y, im);
            j += kw;
            if (j >= W) j -= W;
        }
        R[i] = make_float2(re, im);
    }
    __syncthreads();
    const float norm = rsqrtf((float)HW);
    for (int i = tid; i < np * HWp; i += 256) {
        const int pl = i / HWp, r = i - pl * HWp, kh = r / Wp, kw = r - kh * Wp;
        const float2* col = R + pl * HWp + kw;
        float re = 0.0f, im = 0.0f;
        int j = 0;
        for (int hh = 0; hh < H; ++hh) {
            const float2 t = twH[j], v = col[hh * Wp];
            re = fmaf(v.x, t.x, fmaf(-v.y, t.y, re));
            im = fmaf(v.x, t.y, fmaf(v.y, t.x, im));
            j += kh;
            if (j >= H) j -= H;
        }
        const float sc = norm * (interior_weight(kw, W) > 0.0f ? iscale : 1.0f);
        const size_t base = (size_t)(p0 + pl) * 2 * HWp + r;
        Z[base] = re * sc;
        Z[base + HWp] = im * sc;
    }
}

// Z planes -> y (P, H, W) = irfftn(s=(H,W), ortho) [+ addend]; interior bins x iscale
__global__ __launch_bounds__(256) void irfft2_kernel(const float* __restrict__ Z, int P, int H, int W, int NPW,
                                                     float iscale, const float* __restrict__ addend,
                                                     float* __restrict__ y) {
    extern __shared__ float smem[];
    const int Wp = W / 2 + 1, HWp = H * Wp, HW = H * W;
    float2* twW = reinterpret_cast<float2*>(smem);
    float2* twH = twW + DFT_MAXN;
    float2* Xs = twH + DFT_MAXN;            // NPW * HWp
    float2* R = Xs + NPW * HWp;             // NPW * HWp
    const int tid = threadIdx.x;
    const int p0 = blockIdx.x * NPW;
    const int np = min(NPW, P - p0);
    make_twiddles(twW, W, tid, 256);
    make_twiddles(twH, H, tid, 256);
    for (int i = tid; i < np * HWp; i += 256) {
        const int pl = i / HWp, r = i - pl * HWp;
        const size_t base = (size_t)(p0 + pl) * 2 * HWp + r;
        Xs[i] = make_float2(Z[base], Z[base + HWp]);
    }
    __syncthreads();
    // columns: R[h][kw] = sum_kh X[kh][kw] e^{+2 pi i kh h / H}
    for (int i = tid; i < np * HWp; i += 256) {
        const int pl = i / HWp, r = i - pl * HWp, hh = r / Wp, kw = r - hh * Wp;
        const float2* col = Xs + pl * HWp + kw;
        float re = 0.0f, im = 0.0f;
        int j = 0;
        for (int kh = 0; kh < H; ++kh) {
            const float2 t = twH[j], v = col[kh * Wp];   // conj twiddle: (t.x, -t.y)
            re = fmaf(v.x, t.x, fmaf(v.y, t.y, re));
            im = fmaf(v.y, t.x, fmaf(-v.x, t.y, im));
            j += hh;
            if (j >= H) j -= H;
        }
        const float wgt = interior_weight(kw, W) > 0.0f ? 2.0f * iscale : 1.0f;
        R[i] = make_float2(re * wgt, im * wgt);
    }
    __syncthreads();
    // rows (C2R): y[h][w] = sum_kw Re(R[h][kw] e^{+2 pi i kw w / W}); Im of kw=0, W/2 drops out
    const float norm = rsqrtf((float)HW);
    for (int i = tid; i < np * HW; i += 256) {
        const int pl = i / HW, r = i - pl * HW, hh = r / W, w = r - hh * W;
        const float2* row = R + pl * HWp + hh * Wp;
        float acc = 0.0f;
        int j = 0;
        for (int kw = 0; kw < Wp; ++kw) {
            const float2 t = twW[j], v = row[kw];
            acc = fmaf(v.x, t.x, fmaf(v.y, t.y, acc));   // Re(v * conj(t))
            j += w;
            if (j >= W) j -= W;
        }
        const size_t o = (size_t)(p0 + pl) * HW + r;
        float outv = acc * norm;
        if (addend) outv += addend[o];
        y[o] = outv;
    }
}

// ------------------------------------------------------------------ SELayer backward
// Forward (spectral_transform.py:23-28): m = mean_HW x, h = relu(W1 m), g = sigmoid(W2 h), out = x * g.
// Three launches, so the two plane-wide passes spread over the whole chip (one workgroup per sample
// ran B workgroups: 1 ms per 128x128 fgan128 layer at B = 64):
//   sums  one wave per (b, c) plane: ws.mean = mean_HW x, ws.dot = sum_HW dy * x
//   gate  one workgroup per sample: g, dpre2 = d(W2 h), hact, dpre1 = d(W1 m), dmean = W1^T dpre1 / HW
//   apply dx = dy * g + dmean (per plane), float4 where vec4 (HW % 4 == 0 and x, dout, dx 16-byte aligned)
// ws: 4 * B * C floats (mean, dot, gate, dmean).
__global__ __launch_bounds__(256) void se_bwd_sums_kernel(const float* __restrict__ x, const float* __restrict__ dout,
                                                          int P, int HW, int vec4, float* __restrict__ ws_mean,
                                                          float* __restrict__ ws_dot) {
    const int lane = threadIdx.x & 63;
    const int pl = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (pl >= P) return;
    const float* xp = x + (size_t)pl * HW;
    const float* dp = dout + (size_t)pl * HW;
    float s = 0.0f, q = 0.0f;
    if (vec4) {
        const float4* x4 = reinterpret_cast<const float4*>(xp);
        const float4* d4 = reinterpret_cast<const float4*>(dp);
        for (int i = lane; i < HW / 4; i += 64) {
            const float4 a = x4[i], d = d4[i];
            s += (a.x + a.y) + (a.z + a.w);
            q = fmaf(d.x, a.x, fmaf(d.y, a.y, fmaf(d.z, a.z, fmaf(d.w, a.w, q))));
        }
    } else {
        for (int i = lane; i < HW; i += 64) {
            s += xp[i];
            q = fmaf(dp[i], xp[i], q);
        }
    }
    s = ffc::wave_sum(s);
    q = ffc::wave_sum(q);
    if (lane == 0) {
        ws_mean[pl] = s / (float)HW;
        ws_dot[pl] = q;
    }
}

__global__ __launch_bounds__(256) void se_bwd_gate_kernel(int C, int HW, const float* __restrict__ w1,
                                                          const float* __restrict__ w2, int hid,
                                                          const float* __restrict__ ws_mean,
                                                          const float* __restrict__ ws_dot, float* __restrict__ ws_gate,
                                                          float* __restrict__ ws_dmean, float* __restrict__ dpre2,
                                                          float* __restrict__ hact_o, float* __restrict__ dpre1,
                                                          float* __restrict__ mean_o) {
    extern __shared__ float sm[];
    float* mean = sm;            // C
    float* dot = mean + C;       // C
    float* hpre = dot + C;       // hid (<= 32)
    float* dp1 = hpre + 32;      // hid
    const int b = blockIdx.x, tid = threadIdx.x;
    const size_t o = (size_t)b * C;
    if (hid == 0) {
        for (int c = tid; c < C; c += 256) {
            ws_gate[o + c] = 0.5f;   // Linear(C, 0) -> zeros -> sigmoid(0)
            ws_dmean[o + c] = 0.0f;
        }
        return;
    }
    for (int c = tid; c < C; c += 256) {
        mean[c] = ws_mean[o + c];
        dot[c] = ws_dot[o + c];
    }
    __syncthreads();
    if (tid < hid) {
        float s = 0.0f;
        for (int c = 0; c < C; ++c) s = fmaf(w1[(size_t)tid * C + c], mean[c], s);
        hpre[tid] = s;
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        float s = 0.0f;
        for (int j = 0; j < hid; ++j) s = fmaf(w2[(size_t)c * hid + j], fmaxf(hpre[j], 0.0f), s);
        const float g = 1.0f / (1.0f + expf(-s));
        ws_gate[o + c] = g;
        const float d2 = dot[c] * g * (1.0f - g);
        dot[c] = d2;
        dpre2[o + c] = d2;
        mean_o[o + c] = mean[c];
    }
    __syncthreads();
    if (tid < hid) {
        float s = 0.0f;
        for (int c = 0; c < C; ++c) s = fmaf(w2[(size_t)c * hid + tid], dot[c], s);
        const float d1 = hpre[tid] > 0.0f ? s : 0.0f;
        dp1[tid] = d1;
        dpre1[(size_t)b * hid + tid] = d1;
        hact_o[(size_t)b * hid + tid] = fmaxf(hpre[tid], 0.0f);
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        float s = 0.0f;
        for (int j = 0; j < hid; ++j) s = fmaf(w1[(size_t)j * C + c], dp1[j], s);
        ws_dmean[o + c] = s / (float)HW;
    }
}

__global__ __launch_bounds__(256) void se_bwd_apply_kernel(const float* __restrict__ dout, long long n, int HW,
                                                           int vec4, const float* __restrict__ gate,
                                                           const float* __restrict__ dmean, float* __restrict__ dx) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    if (vec4) {
        const int hw4 = HW / 4;
        const float4* d4 = reinterpret_cast<const float4*>(dout);
        float4* o4 = reinterpret_cast<float4*>(dx);
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += stride) {
            const long long pl = i / hw4;
            const float g = gate[pl], m = dmean[pl];
            const float4 d = d4[i];
            o4[i] = make_float4(fmaf(d.x, g, m), fmaf(d.y, g, m), fmaf(d.z, g, m), fmaf(d.w, g, m));
        }
    } else {
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
            const long long pl = i / HW;
            dx[i] = fmaf(dout[i], gate[pl], dmean[pl]);
        }
    }
}

// ------------------------------------------------------------------ 2x2 pool / x2 nearest upsample
__global__ void pool2_kernel(const float* __restrict__ x, long long P, int H, int W, float scale,
                             float* __restrict__ y) {
    const int h = H / 2, w = W / 2;
    const long long n = P * h * w;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const long long pl = i / ((long long)h * w);
        const int r = (int)(i - pl * h * w), yy = r / w, xx = r - yy * w;
        const float* s = x + (size_t)pl * H * W + (size_t)(2 * yy) * W + 2 * xx;
        y[i] = (s[0] + s[1] + s[W] + s[W + 1]) * scale;
    }
}

__global__ void up2_kernel(const float* __restrict__ x, long long P, int h, int w, float scale,
                           float* __restrict__ y) {
    const int H = 2 * h, W = 2 * w;
    const long long n = P * H * W;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const long long pl = i / ((long long)H * W);
        const int r = (int)(i - pl * H * W), yy = r / W, xx = r - yy * W;
        y[i] = x[(size_t)pl * h * w + (size_t)(yy >> 1) * w + (xx >> 1)] * scale;
    }
}

// ------------------------------------------------------------------ conv onto a 1x1 output, M <= 4
// out[b][m] = act(sum_seg sum_k x_seg[b][k] * w_seg[m][k] + bias[m]): a Conv2d whose kernel covers
// the whole input plane (k == H == W, p = 0), e.g. FFCDiscriminator's last layer (4x4 -> 1x1,
// models/ffc_discriminator.py:31).  One workgroup per sample; a per-sample dot product of K floats.
constexpr int FS_MMAX = 4;

__global__ __launch_bounds__(256) void conv_full_smallm_kernel(const float* __restrict__ x0, int K0,
                                                               const float* __restrict__ w0,
                                                               const float* __restrict__ x1, int K1,
                                                               const float* __restrict__ w1,
                                                               const float* __restrict__ bias, int M,
                                                               float* __restrict__ out, int act, float p) {
    const int b = blockIdx.x, tid = threadIdx.x;
    float acc[FS_MMAX] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int sgi = 0; sgi < 2; ++sgi) {
        const float* x = sgi ? x1 : x0;
        const float* w = sgi ? w1 : w0;
        const int K = sgi ? K1 : K0;
        if (!x) continue;
        const float* xb = x + (size_t)b * K;
        if ((K & 3) == 0) {
            const float4* x4 = reinterpret_cast<const float4*>(xb);
            for (int i = tid; i < K / 4; i += 256) {
                const float4 v = x4[i];
#pragma unroll
                for (int m = 0; m < FS_MMAX; ++m) {
                    if (m >= M) break;
                    const float4 ww = reinterpret_cast<const float4*>(w + (size_t)m * K)[i];
                    acc[m] = fmaf(v.x, ww.x, fmaf(v.y, ww.y, fmaf(v.z, ww.z, fmaf(v.w, ww.w, acc[m]))));
                }
            }
        } else {
            for (int i = tid; i < K; i += 256) {
                const float v = xb[i];
                for (int m = 0; m < M; ++m) acc[m] = fmaf(v, w[(size_t)m * K + i], acc[m]);
            }
        }
    }
    __shared__ float red[4][FS_MMAX];
#pragma unroll
    for (int m = 0; m < FS_MMAX; ++m) {
        const float v = ffc::wave_sum(acc[m]);
        if ((tid & 63) == 0) red[tid >> 6][m] = v;
    }
    __syncthreads();
    if (tid < M) {
        const float v = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid] + (bias ? bias[tid] : 0.0f);
        out[(size_t)b * M + tid] = ffc::apply_act(v, act, p);
    }
}

int grid_for(long long n) { return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192)); }

int dft_npw(int H, int W) { return std::max(1, std::min(64, 1024 / (H * W))); }

size_t dft_lds(int H, int W, int npw, bool inverse) {
    const size_t Wp = W / 2 + 1;
    size_t b = 2 * DFT_MAXN * sizeof(float2);
    if (inverse) b += 2 * (size_t)npw * H * Wp * sizeof(float2);
    else b += (size_t)npw * H * W * sizeof(float) + (size_t)npw * H * Wp * sizeof(float2);
    return b;
}

}  // namespace

extern "C" int ffc_act_bwd(const float* t, const float* dy, float* dx, long long n, int act, float act_param,
                           void* stream) {
    FFC_CHECK_ARG(t && dy && dx && n > 0 && act >= 0 && act <= FFC_ACT_GELU, "ffc_act_bwd: bad args");
    hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, t, dy, dx, n, act,
                       act_param);
    return ffc::launch_status("ffc_act_bwd");
}

extern "C" int ffc_reduce_splits(int B, int C, int HW) {
    // splits per channel so that C * S workgroups fill the chip, each with >= 1024 elements
    const long long per = (long long)B * HW;
    int S = (int)std::max<long long>(1, std::min<long long>(per / 1024, (1024 + C - 1) / C));
    return std::min(S, 256);
}

extern "C" int ffc_channel_moments(const float* x, int B, int C, int HW, double* ws, int S, double* moments,
                                   void* stream) {
    FFC_CHECK_ARG(x && ws && moments && B > 0 && C > 0 && HW > 0 && S > 0, "ffc_channel_moments: bad args");
    hipLaunchKernelGGL(moments_partial_kernel, dim3(C, S), dim3(256), 0, (hipStream_t)stream, x, B, C, HW, S, ws);
    hipLaunchKernelGGL(moments_final_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, ws, S, C,
                       (double)B * HW, moments);
    return ffc::launch_status("ffc_channel_moments");
}

namespace {
// ws[S][C][2] -> sums[C][2] in split order (fixed: deterministic)
__global__ void bn_bwd_sums_kernel(const double* __restrict__ ws, int S, int C, double* __restrict__ sums) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double a = 0.0, b = 0.0;
    for (int s = 0; s < S; ++s) {
        a += ws[((size_t)s * C + c) * 2];
        b += ws[((size_t)s * C + c) * 2 + 1];
    }
    sums[2 * c] = a;
    sums[2 * c + 1] = b;
}
}  // namespace

// SyncBN backward in three steps (the caller all-reduces the sums in between)
extern "C" int ffc_bn_bwd_sums(const float* x, const float* dy, int B, int C, int HW, const float* scale,
                               const float* shift, int act, float act_param, double* ws, int S, double* sums,
                               void* stream) {
    FFC_CHECK_ARG(x && dy && scale && shift && ws && sums && B > 0 && C > 0 && HW > 0 && S > 0,
                  "ffc_bn_bwd_sums: bad args");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(bn_bwd_partial_kernel, dim3(C, S), dim3(256), 0, s, x, dy, B, C, HW, S, scale, shift, act,
                       act_param, ws);
    hipLaunchKernelGGL(bn_bwd_sums_kernel, dim3((C + 255) / 256), dim3(256), 0, s, ws, S, C, sums);
    return ffc::launch_status("ffc_bn_bwd_sums");
}

extern "C" int ffc_bn_bwd_coeff(const double* sums, int C, const double* moments, float eps, const float* gamma,
                                float* coef, float* dgamma, float* dbeta, void* stream) {
    FFC_CHECK_ARG(sums && moments && coef && C > 0, "ffc_bn_bwd_coeff: bad args");
    hipLaunchKernelGGL(bn_bwd_coeff_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, 1, C,
                       moments, nullptr, nullptr, eps, gamma, coef, dgamma, dbeta);
    return ffc::launch_status("ffc_bn_bwd_coeff");
}

extern "C" int ffc_bn_bwd_apply(const float* x, const float* dy, int B, int C, int HW, const float* scale,
                                const float* shift, int act, float act_param, const float* coef, float* dx,
                                void* stream) {
    FFC_CHECK_ARG(x && dy && scale && shift && coef && dx && B > 0 && C > 0 && HW > 0, "ffc_bn_bwd_apply: bad args");
    const long long total = (long long)B * C * HW;
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, dy, C, HW,
                       total, scale, shift, act, act_param, coef, dx);
    return ffc::launch_status("ffc_bn_bwd_apply");
}

extern "C" int ffc_bn_bwd(const float* x, const float* dy, int B, int C, int HW, const float* scale,
                          const float* shift, int act, float act_param, const double* moments, const float* rmean,
                          const float* rvar, float eps, const float* gamma, double* ws, int S, float* coef,
                          float* dgamma, float* dbeta, float* dx, void* stream) {
    FFC_CHECK_ARG(x && dy && scale && shift && ws && coef && B > 0 && C > 0 && HW > 0 && S > 0,
                  "ffc_bn_bwd: bad args");
    FFC_CHECK_ARG(moments || (rmean && rvar), "ffc_bn_bwd: need batch moments or running stats");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(bn_bwd_partial_kernel, dim3(C, S), dim3(256), 0, s, x, dy, B, C, HW, S, scale, shift, act,
                       act_param, ws);
    hipLaunchKernelGGL(bn_bwd_coeff_kernel, dim3((C + 255) / 256), dim3(256), 0, s, ws, S, C, moments, rmean, rvar,
                       eps, gamma, coef, dgamma, dbeta);
    if (dx) {
        const long long total = (long long)B * C * HW;
        hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, dy, C, HW, total, scale,
                           shift, act, act_param, coef, dx);
    }
    return ffc::launch_status("ffc_bn_bwd");
}

extern "C" int ffc_conv_wgrad_tile(int Mu, int NT) { return wgrad_tile(Mu, NT); }

extern "C" int ffc_conv_wgrad(const float* U, int Mu, int PH, int PW, const float* V, int Nv, int VH, int VW, int B,
                              int k, int stride, int pad, int dil, int S, float* ws, float* dW, int accumulate,
                              void* stream) {
    FFC_CHECK_ARG(U && V && dW && Mu > 0 && Nv > 0 && PH > 0 && PW > 0 && VH > 0 && VW > 0 && B > 0 && k > 0 &&
                      stride > 0 && dil > 0 && S >= 1 && (long long)S <= (long long)B * PH * PW,
                  "ffc_conv_wgrad: bad args");
    FFC_CHECK_ARG(S == 1 || ws, "ffc_conv_wgrad: split-K needs a workspace");
    const int NT = Nv * k * k;
    WgradArgs a{U, V, (S == 1 && !accumulate) ? dW : ws, B, Mu, PH, PW, Nv, VH, VW, k, stride, pad, dil, S};
    FFC_CHECK_ARG(a.out, "ffc_conv_wgrad: accumulate needs a workspace");
    const int bt = wgrad_tile(Mu, NT);
    dim3 grid((NT + bt - 1) / bt, (Mu + bt - 1) / bt, S);
    static const int bk_knob = [] {   // A/B measurement knob (tools/wgrad_probe.py): K chunk depth
        const char* e = getenv("FFC_WGRAD_BK");
        return e ? atoi(e) : 0;
    }();
    static const bool exact = [] {    // A/B knob: f32-input MFMA instead of the split-bf16 products
        const char* e = getenv("FFC_WGRAD_ARITH");
        return e && std::string(e) == "f32";
    }();
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(256), 0, (hipStream_t)stream, a); };
    const char* kv = getenv("FFC_WGRAD_KERNEL");   // A/B knob: "old" = the split-per-use kernel below
    if (!exact && !bk_knob && !(kv && std::string(kv) == "old")) {
        bt == 128 ? go(wgradq_kernel<128, 128>) : go(wgradq_kernel<64, 64>);
    } else if (bt == 128) {   // 32-deep chunks: 64 MFMAs per wave between barriers (measured 18 % faster than 16)
        if (bk_knob == 16)
            exact ? go(wgrad_kernel<128, 16, false>) : go(wgrad_kernel<128, 16, true>);
        else
            exact ? go(wgrad_kernel<128, 32, false>) : go(wgrad_kernel<128, 32, true>);
    } else {   // 64-deep chunks (32 measured slower: the small tile needs the deeper load batch)
        if (bk_knob == 32)
            exact ? go(wgrad_kernel<64, 32, false>) : go(wgrad_kernel<64, 32, true>);
        else
            exact ? go(wgrad_kernel<64, 64, false>) : go(wgrad_kernel<64, 64, true>);
    }
    if (a.out != dW) {
        const long long n = (long long)Mu * NT;
        if (n >= 65536 || S < 32)
            hipLaunchKernelGGL(split_sum_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, ws, S, n, dW,
                               accumulate);
        else
            hipLaunchKernelGGL(split_sum_grouped_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                               (hipStream_t)stream, ws, S, n, dW, accumulate);
    }
    return ffc::launch_status("ffc_conv_wgrad");
}

extern "C" int ffc_rfft2_planes(const float* x, int P, int H, int W, float interior_scale, float* Z, void* stream) {
    FFC_CHECK_ARG(x && Z && P > 0 && H >= 1 && W >= 2, "ffc_rfft2_planes: bad args");
    // square power-of-two planes 8..128: line FFTs (fu2d_kernels.hip); others: direct DFT up to 64
    if (H >= 8 && H == W && (H & (H - 1)) == 0) {
        const int rc = ffc::fft_planes_r2c(x, P, H, W, interior_scale, Z, stream);
        if (rc != 1) return rc;
    }
    FFC_CHECK_ARG(H <= DFT_MAXN && W <= DFT_MAXN,
                  "ffc_rfft2_planes: planes up to 64x64 (square powers of two up to 128x128)");
    const int npw = dft_npw(H, W);
    hipLaunchKernelGGL(rfft2_kernel, dim3((P + npw - 1) / npw), dim3(256), dft_lds(H, W, npw, false),
                       (hipStream_t)stream, x, P, H, W, npw, interior_scale, Z);
    return ffc::launch_status("ffc_rfft2_planes");
}

extern "C" int ffc_irfft2_planes(const float* Z, int P, int H, int W, float interior_scale, const float* addend,
                                 float* y, void* stream) {
    FFC_CHECK_ARG(Z && y && P > 0 && H >= 1 && W >= 2, "ffc_irfft2_planes: bad args");
    if (H >= 16 && H == W && (H & (H - 1)) == 0) {
        const int rc = ffc::fft_planes_c2r(Z, P, H, W, interior_scale, addend, y, stream);
        if (rc != 1) return rc;
    }
    FFC_CHECK_ARG(H <= DFT_MAXN && W <= DFT_MAXN,
                  "ffc_irfft2_planes: planes up to 64x64 (square powers of two up to 128x128)");
    const int npw = dft_npw(H, W);
    hipLaunchKernelGGL(irfft2_kernel, dim3((P + npw - 1) / npw), dim3(256), dft_lds(H, W, npw, true),
                       (hipStream_t)stream, Z, P, H, W, npw, interior_scale, addend, y);
    return ffc::launch_status("ffc_irfft2_planes");
}

extern "C" int ffc_se_bwd(const float* x, const float* dout, int B, int C, int H, int W, const float* w1,
                          const float* w2, int hidden, float* dx, float* dpre2, float* hact, float* dpre1, float* mean,
                          float* ws, void* stream) {
    FFC_CHECK_ARG(x && dout && dx && ws && B > 0 && C > 0 && H > 0 && W > 0 && hidden >= 0 && hidden <= 32,
                  "ffc_se_bwd: bad args");
    FFC_CHECK_ARG(hidden == 0 || (w1 && w2 && dpre2 && hact && dpre1 && mean), "ffc_se_bwd: missing buffers");
    const size_t lds = (2 * (size_t)C + 64) * sizeof(float);
    FFC_CHECK_ARG(lds <= 64 * 1024, "ffc_se_bwd: too many channels");
    const int P = B * C, HW = H * W;
    float* ws_mean = ws;
    float* ws_dot = ws + P;
    float* ws_gate = ws + 2 * (size_t)P;
    float* ws_dmean = ws + 3 * (size_t)P;
    hipStream_t s = (hipStream_t)stream;
    // float4 planes only where every plane starts 16-byte aligned (an offset pointer takes the scalar loops)
    const int vec4 = (HW & 3) == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dout) |
                                        reinterpret_cast<uintptr_t>(dx)) & 15) == 0;
    if (hidden > 0)
        hipLaunchKernelGGL(se_bwd_sums_kernel, dim3((P + 3) / 4), dim3(256), 0, s, x, dout, P, HW, vec4, ws_mean,
                           ws_dot);
    hipLaunchKernelGGL(se_bwd_gate_kernel, dim3(B), dim3(256), lds, s, C, HW, w1, w2, hidden, ws_mean, ws_dot,
                       ws_gate, ws_dmean, dpre2, hact, dpre1, mean);
    const long long n = (long long)P * HW;
    const long long units = vec4 ? n / 4 : n;
    const int grid = (int)std::min<long long>((units + 255) / 256, 8192);
    hipLaunchKernelGGL(se_bwd_apply_kernel, dim3(grid), dim3(256), 0, s, dout, n, HW, vec4, ws_gate, ws_dmean, dx);
    return ffc::launch_status("ffc_se_bwd");
}

extern "C" int ffc_conv_full_smallm(const float* x0, int K0, const float* w0, const float* x1, int K1,
                                    const float* w1, const float* bias, int B, int M, float* out, int act,
                                    float act_param, void* stream) {
    FFC_CHECK_ARG(x0 && w0 && out && B > 0 && K0 > 0 && M >= 1 && M <= FS_MMAX, "ffc_conv_full_smallm: bad args");
    FFC_CHECK_ARG(!x1 || (w1 && K1 > 0), "ffc_conv_full_smallm: second segment");
    const bool al = ((reinterpret_cast<uintptr_t>(x0) | reinterpret_cast<uintptr_t>(w0)) & 15) == 0 &&
                    (!x1 || ((reinterpret_cast<uintptr_t>(x1) | reinterpret_cast<uintptr_t>(w1)) & 15) == 0);
    FFC_CHECK_ARG(al, "ffc_conv_full_smallm: 16-byte aligned operands");
    hipLaunchKernelGGL(conv_full_smallm_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, x0, K0, w0, x1, K1, w1,
                       bias, M, out, act, act_param);
    return ffc::launch_status("ffc_conv_full_smallm");
}

extern "C" int ffc_pool2(const float* x, long long P, int H, int W, float scale, float* y, void* stream) {
    FFC_CHECK_ARG(x && y && P > 0 && H >= 2 && W >= 2 && H % 2 == 0 && W % 2 == 0, "ffc_pool2: bad args");
    hipLaunchKernelGGL(pool2_kernel, dim3(grid_for(P * H * W / 4)), dim3(256), 0, (hipStream_t)stream, x, P, H, W,
                       scale, y);
    return ffc::launch_status("ffc_pool2");
}

extern "C" int ffc_up2(const float* x, long long P, int h, int w, float scale, float* y, void* stream) {
    FFC_CHECK_ARG(x && y && P > 0 && h > 0 && w > 0, "ffc_up2: bad args");
    hipLaunchKernelGGL(up2_kernel, dim3(grid_for(P * h * w * 4)), dim3(256), 0, (hipStream_t)stream, x, P, h, w,
                       scale, y);
    return ffc::launch_status("ffc_up2");
}
