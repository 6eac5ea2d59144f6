// LDS-patch implicit-GEMM convolution for gfx950 (MFMA, fp32-accurate) — the local-branch hot path.
//
// Replaces nn.ConvTranspose2d / nn.Conv2d of FFCTranspose / FFC (layers/ffc/ffc_transpose.py:79-86,
// layers/ffc/ffc.py:45-70) together with SpectralTransform.conv2 (spectral_transform.py:70-71,108),
// which is folded in as a 1x1 segment at the output resolution.
//
// Work decomposition (one workgroup = 4 waves):
//   * 32 output channels (M-tile) x a pixel block (NS samples x TR x TC pixels of the phase grid)
//   * NP = 4 (stride-2 transposed conv): wave w computes phase w = (py, px) of every pixel of the
//     block; NP = 1 (direct conv): the waves split the pixel block.
//   * K runs over (segment, chunk, tap), a chunk being 16 channels (segments with 1, 2 or 4 taps
//     per phase) or 4 channels x 16 taps (Conv2d k4 s2, one phase).  Per chunk the input patch the block needs is
//     staged once in LDS (zero outside the input, 2x2 avg-pool / SE gate applied on the way in);
//     every (phase, tap) B fragment is a conflict-free ds_read_b32 from it.  The next chunk's
//     global loads are in flight (registers) while the current chunk's MFMAs run.
//   * A (packed weights, k = (seg, ch, tap), each 16-k group of one lane half contiguous) is read
//     straight from L2 as 2 x dwordx4 per lane per 16 k and shared by the wave's N-tiles.
//   * Products: by default fp32-accurate split-bf16 MFMA (split3 / mfma_split3 below: 6 x
//     v_mfma_f32_32x32x16_bf16 per 16 k); cfg | FFC_CONVP_EXACT_F32 runs v_mfma_f32_32x32x2_f32
//     (bitwise fp32 fma chains).  Lane half h of k-step s carries k = 16g + 8h + s in both.
#include "ffc_internal.h"

#include <string>

namespace {

struct ConvPArgs {
    ffc_convp_job jobs[2];
    const int4* tiles;
    int ebuf;                      // floats per LDS patch buffer (multiple of 256)
};

__device__ float g_zero_src[64];   // source of the zero fill for out-of-bounds patch elements

#ifdef FFC_TRACE
// Diagnostic build only (tools/trace_convp.py): per workgroup {realtime start, end, HW_ID | XCC_ID << 32,
// wave-0 cycles in barrier / staging issue / MFMA section, total cycles, chunks}.
__device__ unsigned long long g_ffc_trace[8 * 4096];
#define FFC_STAMP(t)                                                                        \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                  \
    } while (0)
#endif

typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;


constexpr int NEMAX = 8;   // staging units (4-float groups, or floats) per thread per chunk

// split3 / mfma_split3 (fp32-accurate products on the bf16 MFMA): ffc_internal.h

// Per-segment staging state: the chunk-invariant part of every unit this thread moves.
// Unit n of the patch image [ns][ch][pr][col] (col in 4-float groups when vec4) maps to
// x + off[e] + ch0 * IH*IW; off < 0 marks a unit outside the input / batch (zero fill).
struct Stager {
    const float* x;
    int C, Cpad, IHW, T, kseg, vec4, nunits, cc, lcc;
    int off[NEMAX];
    unsigned chn;   // 4-bit channel-in-chunk of each of the thread's units
};

// A row pointer + patch geometry for the segment whose chunks are being multiplied.
struct Computer {
    int T, lt, PRC, gstep, Cpad, cc;
    int sb[8];      // per k-step s8: (s8 >> lt) * PRC + tap offset (s8 & (T-1))
};

// AR: 0 = f32-input MFMA, 1 = split-bf16 (A split in registers), 2 = split-bf16 with A pre-split
// (ffc_convp_job.A3 planes)
template <int NP, int NTW, int AR>
__global__ __launch_bounds__(256) void convp_kernel(ConvPArgs args_byval) {
#if defined(__HIP_DEVICE_COMPILE__)
    const ConvPArgs& args = *(const ConvPArgs*)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const ConvPArgs& args = args_byval;
#endif
    constexpr bool SPLIT = AR > 0;
    extern __shared__ __attribute__((aligned(16))) float patch[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5, cl = lane & 31;
    const int4 tile = args.tiles[blockIdx.x];
    const int ji = __builtin_amdgcn_readfirstlane(tile.x);
    const int m0 = __builtin_amdgcn_readfirstlane(tile.y);
    const int pb = __builtin_amdgcn_readfirstlane(tile.z);
    const ffc_convp_job& J = args.jobs[ji];
    const int p = NP == 4 ? wave : 0;
    const ffc_convp_phase& P = J.ph[p];
    const int ebuf = args.ebuf;

    const int NS = J.NS, TR = J.TR, TC = J.TC;
    const int bs = pb / (J.nrb * J.ncb);
    const int prem = pb - bs * J.nrb * J.ncb;
    const int rb = prem / J.ncb, cb = prem - rb * J.ncb;
    const int b0 = bs * NS, r0 = rb * TR, c0 = cb * TC;
    const int TRC = TR * TC;
    const int nseg = J.nseg;

    // this lane's pixels (one per N-tile)
    int pns[NTW], pr_[NTW], pc_[NTW];
    bool pv[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
        const int q = ((NP == 4 ? 0 : wave * NTW) + nt) * 32 + cl;
        const int ns = q / TRC;
        const int rem = q - ns * TRC;
        const int r = rem / TC, c = rem - r * TC;
        pns[nt] = ns;
        pr_[nt] = r;
        pc_[nt] = c;
        pv[nt] = ns < NS && b0 + ns < J.B && r0 + r < P.PH && c0 + c < P.PW;
    }

    floatx16 acc[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[nt][r] = 0.0f;

    // ---- staging: segment geometry (once per segment, not per chunk)
    const float* zsrc = g_zero_src;
    asm volatile("" : "+s"(zsrc));   // keep the zero-fill source in SGPRs (no per-unit GOT reload)
    Stager st;
    auto stage_setup = [&](int s) {
        const ffc_convp_seg& S = J.seg[s];
        st.x = S.x;
        st.C = S.C;
        st.Cpad = S.Cpad;
        st.IHW = S.IH * S.IW;
        st.T = P.T[s];
        st.kseg = P.kseg[s];
        st.vec4 = S.vec4;
        st.cc = S.cc;
        st.lcc = S.cc == 4 ? 2 : 4;
        const int PR = S.PR;
        const int iy0 = r0 * S.mult_y + S.org_y;
        const int ix0 = c0 * S.mult_x + S.org_x;
        const int xa = S.vec4 ? (ix0 & ~3) : ix0;
        const int PCu = S.vec4 ? S.PC / 4 : S.PC;   // units per patch row (4-float groups when vec4)
        const int step = S.vec4 ? 4 : 1;
        st.nunits = NS * st.cc * PR * PCu;
        st.chn = 0;
        // n / d as umulhi(n, ceil(2^32 / d)): exact for n < 2^16 (n < 2048 units here); d = 1 special
        const unsigned mPC = PCu > 1 ? 0xFFFFFFFFu / (unsigned)PCu + 1u : 0u;
        const unsigned mPR = PR > 1 ? 0xFFFFFFFFu / (unsigned)PR + 1u : 0u;
#pragma unroll
        for (int e = 0; e < NEMAX; ++e) {
            const unsigned n = (unsigned)(e * 256 + tid);
            const unsigned q1 = PCu > 1 ? __umulhi(n, mPC) : n;
            const int g = (int)(n - q1 * PCu);
            const unsigned q2 = PR > 1 ? __umulhi(q1, mPR) : q1;
            const int pr = (int)(q1 - q2 * PR);
            const int ns = (int)(q2 >> st.lcc), ch = (int)(q2 & (st.cc - 1));
            const int b = b0 + ns, iy = iy0 + pr, ix = xa + g * step;
            const bool ok = (int)n < st.nunits && b < J.B && (unsigned)iy < (unsigned)S.IH &&
                            (unsigned)ix < (unsigned)S.IW;
            st.off[e] = ok ? ((b * S.C + ch) * S.IH + iy) * S.IW + ix : -1;
            st.chn |= (unsigned)ch << (4 * e);
        }
    };
    // LDS-DMA of one chunk: unit n -> lane n % 64 of wave-instruction n / 64 (no VGPR staging)
    auto stage_issue = [&](int ch0, float* dst) {
        const int cmax = st.C - ch0;
        const float* xb = st.x + ch0 * st.IHW;
        const int nw = (st.nunits + 255) >> 8;
        if (st.vec4) {
#pragma unroll
            for (int e = 0; e < NEMAX; ++e) {
                if (e < nw) {
                    const bool ok = st.off[e] >= 0 && (int)((st.chn >> (4 * e)) & 15) < cmax;
                    const float* src = ok ? xb + st.off[e] : zsrc;
                    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (e * 256 + wave * 64) * 4), 16, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < NEMAX; ++e) {
                if (e < nw) {
                    const bool ok = st.off[e] >= 0 && (int)((st.chn >> (4 * e)) & 15) < cmax;
                    const float* src = ok ? xb + st.off[e] : zsrc;
                    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + e * 256 + wave * 64), 4, 0, 0);
                }
            }
        }
    };
    // A of one chunk (4 groups of 16 k; groups >= min(T, 4) are loaded but unused: the packed
    // buffer carries tail padding) into registers, not waited for here
    auto load_A = [&](int ch0, floatx4 (&n0)[4], floatx4 (&n1)[4]) {
        const float* __restrict__ Ap =
            J.A + P.a_off + (size_t)(m0 + cl) * P.Kpad + st.kseg + ch0 * st.T + 8 * h;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            n0[g] = *reinterpret_cast<const floatx4*>(Ap + 16 * g);
            n1[g] = *reinterpret_cast<const floatx4*>(Ap + 16 * g + 4);
        }
    };

    // the same A rows from the three pre-split bf16 planes: 8 consecutive k per lane = one dwordx4
    auto load_A3 = [&](int ch0, u32x4 (&n)[3][4]) {
        const uint16_t* __restrict__ Ap =
            J.A3 + P.a_off + (size_t)(m0 + cl) * P.Kpad + st.kseg + ch0 * st.T + 8 * h;
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                n[q][g] = *reinterpret_cast<const u32x4*>(Ap + q * J.a3_stride + 16 * g);
    };

    // ---- compute: per-segment LDS read offsets
    Computer cp;
    int lb[NTW];   // per N-tile byte offset of the lane's pixel inside a chunk buffer (+ lane-half channel)
    auto compute_setup = [&](int s) {
        const ffc_convp_seg& S = J.seg[s];
        const int T = P.T[s];
        cp.T = T;
        cp.Cpad = S.Cpad;
        cp.cc = S.cc;
        if (T == 0) return;
        cp.lt = T == 16 ? 4 : (T == 4 ? 2 : (T == 2 ? 1 : 0));   // k = (channel, tap): tap = k & (T - 1)
        const int PCa = S.PC;
        const int ix0 = c0 * S.mult_x + S.org_x;
        const int xoff = S.vec4 ? ix0 - (ix0 & ~3) : 0;
        cp.PRC = S.PR * PCa;
        cp.gstep = (16 >> cp.lt) * cp.PRC;
        int tap[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int tt = P.tap[s][t & (T - 1)];
            tap[t] = (tt >> 16) * PCa + (tt & 0xFFFF);
        }
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) cp.sb[s8] = (s8 >> cp.lt) * cp.PRC + tap[s8 & (T - 1)];
        // lane half h carries k = 16g + 8h + s8: 8h / T channels further on (T <= 4), or taps 8..15 (T = 16)
        const int th = P.tap_h[s];
        const int hoff = ((8 * h) >> cp.lt) * cp.PRC + (T == 16 ? h * ((th >> 16) * PCa + (th & 0xFFFF)) : 0);
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
            lb[nt] = 4 * (pns[nt] * (cp.cc * cp.PRC) + pr_[nt] * S.mult_y * PCa + pc_[nt] * S.mult_x + xoff + hoff);
    };

    int nchunks = 0;
    for (int s = 0; s < nseg; ++s) nchunks += J.seg[s].Cpad / J.seg[s].cc;

#ifdef FFC_TRACE
    unsigned long long tr_rt0 = __builtin_amdgcn_s_memrealtime(), tr_c0, tr_a, tr_b, tr_bar = 0, tr_stg = 0, tr_mf = 0;
    FFC_STAMP(tr_c0);
#endif
    // stager runs one chunk ahead of the computer
    int ss = 0, sch = 0;   // segment / channel offset of the next chunk to stage
    int cs = 0, cch = 0;   // ... of the chunk being multiplied
    stage_setup(0);
    compute_setup(0);
    floatx4 a0[4], a1[4], n0[4], n1[4];
    u32x4 c3[3][4], n3[3][4];   // AR == 2: current / next chunk's A planes
    stage_issue(0, patch);
    if constexpr (AR == 2)
        load_A3(0, n3);
    else
        load_A(0, n0, n1);
    sch = st.cc;
    if (sch >= st.Cpad && nseg > 1) {
        ss = 1;
        sch = 0;
        stage_setup(1);
    }
#ifdef FFC_TRACE
    unsigned long long tr_ls, tr_le;
    FFC_STAMP(tr_ls);
#endif
    for (int ci = 0; ci < nchunks; ++ci) {
#ifdef FFC_TRACE
        FFC_STAMP(tr_a);
#endif
        __syncthreads();  // patch + A of chunk ci landed (vmcnt(0)); everyone is done with chunk ci-1
#ifdef FFC_TRACE
        FFC_STAMP(tr_b);
        tr_bar += tr_b - tr_a;
#endif
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if constexpr (AR == 2) {
                c3[0][g] = n3[0][g];
                c3[1][g] = n3[1][g];
                c3[2][g] = n3[2][g];
            } else {
                a0[g] = n0[g];
                a1[g] = n1[g];
            }
        }
        if (ci + 1 < nchunks) {  // next chunk's A and patch stay in flight under this chunk's MFMAs
#ifndef FFC_PROBE_NOA   // timing-probe builds only (wrong results): drop the A loads / patch staging
            if constexpr (AR == 2)
                load_A3(sch, n3);
            else
                load_A(sch, n0, n1);
#endif
#ifndef FFC_PROBE_NOSTAGE
            stage_issue(sch, patch + ((ci + 1) & 1) * ebuf);
#endif
            sch += st.cc;
            if (sch >= st.Cpad && ss + 1 < nseg) {
                ++ss;
                sch = 0;
                stage_setup(ss);
            }
        }
#ifdef FFC_TRACE
        FFC_STAMP(tr_a);
        tr_stg += tr_a - tr_b;
#endif
        const int T = cp.T;
#ifndef FFC_PROBE_NOMFMA
        if (T > 0) {
            const int base = ((ci & 1) * ebuf) * 4;   // byte offset of this chunk's buffer
            if constexpr (SPLIT) {
                // one 32x32x16 k-step per (group, N-tile): element j of lane half h is k = 16g + 8h + j,
                // the same k order as the f32 path's k-steps (bf16 A/B lane maps).  The B reads of
                // the next (group, N-tile) are issued before this one's split + MFMAs.
                const int ng = T == 16 ? 4 : T;
                auto rd = [&](int g, int nt, float (&b)[8]) {
                    const int gb = base + 4 * g * cp.gstep + lb[nt];
#pragma unroll
                    for (int s8 = 0; s8 < 8; ++s8)
                        b[s8] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(patch) +
                                                                (gb + 4 * cp.sb[s8]));
                };
#ifdef FFC_CONVP_NO_PREFETCH   // A/B measurement builds
                constexpr bool PF = false;
#else
                constexpr bool PF = true;
#endif
                float bq[2][8];
                if (PF) rd(0, 0, bq[0]);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (g < ng) {
                        Split3 as;
                        if constexpr (AR == 2) {
                            as.hi = __builtin_bit_cast(bf16x8, c3[0][g]);
                            as.mid = __builtin_bit_cast(bf16x8, c3[1][g]);
                            as.lo = __builtin_bit_cast(bf16x8, c3[2][g]);
                        } else {
                            const float av[8] = {a0[g][0], a0[g][1], a0[g][2], a0[g][3],
                                                 a1[g][0], a1[g][1], a1[g][2], a1[g][3]};
                            as = split3(av);
                        }
#pragma unroll
                        for (int nt = 0; nt < NTW; ++nt) {
                            const int cur = PF ? (g * NTW + nt) & 1 : 0;
                            if (!PF)
                                rd(g, nt, bq[cur]);
                            else if (nt + 1 < NTW)
                                rd(g, nt + 1, bq[cur ^ 1]);
                            else if (g + 1 < ng)
                                rd(g + 1, 0, bq[cur ^ 1]);
                            acc[nt] = mfma_split3(as, split3(bq[cur]), acc[nt]);
                        }
                    }
                }
            } else {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (g < T || T == 16) {
                        const float av[8] = {a0[g][0], a0[g][1], a0[g][2], a0[g][3],
                                             a1[g][0], a1[g][1], a1[g][2], a1[g][3]};
                        const int gb = base + 4 * g * cp.gstep;
#pragma unroll
                        for (int s8 = 0; s8 < 8; ++s8) {
                            const int sb = gb + 4 * cp.sb[s8];
#pragma unroll
                            for (int nt = 0; nt < NTW; ++nt) {
                                const float bv = *reinterpret_cast<const float*>(
                                    reinterpret_cast<const char*>(patch) + (lb[nt] + sb));
                                acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s8], bv, acc[nt], 0, 0, 0);
                            }
                        }
                    }
                }
            }
        }
#endif
#ifdef FFC_TRACE
        FFC_STAMP(tr_b);
        tr_mf += tr_b - tr_a;
#endif
        cch += cp.cc;
        if (cch >= cp.Cpad && cs + 1 < nseg) {
            ++cs;
            cch = 0;
            compute_setup(cs);
        }
    }
#ifdef FFC_TRACE
    FFC_STAMP(tr_le);
#endif

    // ---------------- epilogue: bias/addend, BN partials, activation, store
    // The job fields are copied out of the kernel-argument struct first: the compiler cannot tell that
    // the output / slab stores leave the argument memory alone and reloaded every field read through J
    // after each store (an s_load + s_waitcnt per stored element, r04 ISA).
    float* const eout = J.out;
    const float* const ebias = J.bias;
    const float* const eadd = J.addend;
    float* const estats = J.stats;
    const int eM = J.M;
    const size_t plane = (size_t)J.OH * J.OW;
    long long obase[NTW];   // per N-tile: element offset of (sample, channel 0, pixel)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
        obase[nt] = (long long)(b0 + pns[nt]) * eM * (long long)plane +
                    ((r0 + pr_[nt]) * J.Sy + P.py) * J.OW + ((c0 + pc_[nt]) * J.Sx + P.px);
    const int mbase = m0 + 4 * h;
    if (ebias || eadd) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + (r & 3) + 8 * (r >> 2);
            if (m >= eM) continue;
            const float bv = ebias ? ebias[m] : 0.0f;
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
                float v = acc[nt][r] + bv;
                if (eadd && pv[nt]) v += eadd[obase[nt] + (long long)m * plane];
                acc[nt][r] = v;
            }
        }
    }
    if (estats) {
        float cntl = 0.0f;
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) cntl += pv[nt] ? 1.0f : 0.0f;
        const float cnt = ffc::half_wave_sum(cntl);
        float4* stp = reinterpret_cast<float4*>(estats) + ((size_t)pb * 4 + wave) * eM;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + (r & 3) + 8 * (r >> 2);
            float s = 0.0f;
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) s += pv[nt] ? acc[nt][r] : 0.0f;
            const float mean = cnt > 0.0f ? ffc::half_wave_sum(s) / cnt : 0.0f;
            float q = 0.0f;
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
                const float d = pv[nt] ? acc[nt][r] - mean : 0.0f;
                q += d * d;
            }
            const float m2 = ffc::half_wave_sum(q);
            if (cl == 0 && m < eM) stp[m] = make_float4(cnt, mean, m2, 0.0f);
        }
    }
    auto store = [&](auto actf) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + (r & 3) + 8 * (r >> 2);
            if (m < eM) {
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt)
                    if (pv[nt]) eout[obase[nt] + (long long)m * plane] = actf(acc[nt][r]);
            }
        }
    };
    const float ap = J.act_param;
    switch (J.act) {
        case FFC_ACT_RELU: store([](float v) { return fmaxf(v, 0.0f); }); break;
        case FFC_ACT_LEAKY_RELU: store([ap](float v) { return v > 0.0f ? v : v * ap; }); break;
        case FFC_ACT_TANH: store([](float v) { return tanhf(v); }); break;
        case FFC_ACT_SIGMOID: store([](float v) { return 1.0f / (1.0f + expf(-v)); }); break;
        case FFC_ACT_GELU: store([](float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }); break;
        default: store([](float v) { return v; }); break;
    }
#ifdef FFC_TRACE
    __syncthreads();
    unsigned long long tr_c1;
    FFC_STAMP(tr_c1);
    if (tid == 0) {
        unsigned long long* t = g_ffc_trace + 8 * blockIdx.x;
        t[0] = tr_rt0;
        t[1] = __builtin_amdgcn_s_memrealtime();
        t[2] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
               ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
        t[3] = tr_bar;
        t[4] = tr_stg;
        t[5] = tr_mf;
        t[6] = tr_c1 - tr_c0;
        t[7] = (tr_ls - tr_c0) | ((tr_c1 - tr_le) << 32);   // prologue | epilogue cycles
    }
#endif
}

template <int NP, int NTW, int AR>
int launch(const ConvPArgs& a, int ntiles, size_t lds, hipStream_t s) {
    auto k = convp_kernel<NP, NTW, AR>;
    if (lds > 64 * 1024) {
        static bool raised = false;  // per instantiation
        if (!raised) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) {
                ffc::set_error(std::string("ffc_convp_forward: hipFuncSetAttribute: ") + hipGetErrorString(e));
                return FFC_E_LAUNCH;
            }
            raised = true;
        }
    }
    hipLaunchKernelGGL(k, dim3(ntiles), dim3(256), lds, s, a);
    return ffc::launch_status("ffc_convp_forward");
}

}  // namespace

#ifdef FFC_TRACE
extern "C" int ffc_debug_trace_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_ffc_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int ffc_convp_forward(const ffc_convp_job* jobs, int njobs, const int* tiles, int ntiles, int cfg,
                                 void* stream) {
    FFC_CHECK_ARG(jobs && tiles && njobs >= 1 && njobs <= 2 && ntiles > 0, "ffc_convp_forward: bad args");
    const bool exact = (cfg & FFC_CONVP_EXACT_F32) != 0;
    cfg &= ~FFC_CONVP_EXACT_F32;
    size_t emax = 0;
    const int np = (cfg <= 1) ? 4 : 1;
    for (int j = 0; j < njobs; ++j) {
        const ffc_convp_job& J = jobs[j];
        FFC_CHECK_ARG(J.A && J.out && J.B > 0 && J.M > 0, "ffc_convp_forward: incomplete job");
        FFC_CHECK_ARG(J.nphase == np, "ffc_convp_forward: phase count does not match cfg");
        FFC_CHECK_ARG(J.nseg >= 1 && J.nseg <= FFC_MAX_SEG, "ffc_convp_forward: nseg out of range");
        FFC_CHECK_ARG(J.Mpad % 128 == 0 && J.Mpad >= J.M, "ffc_convp_forward: Mpad");
        FFC_CHECK_ARG(J.NS > 0 && J.TR > 0 && J.TC > 0 && J.nrb > 0 && J.ncb > 0, "ffc_convp_forward: tiling");
        for (int s = 0; s < J.nseg; ++s) {
            const ffc_convp_seg& S = J.seg[s];
            FFC_CHECK_ARG(S.cc == 16 || (S.cc == 4 && J.nphase == 1), "ffc_convp_forward: channels per chunk");
            FFC_CHECK_ARG(S.x && S.Cpad % S.cc == 0 && S.Cpad >= S.C, "ffc_convp_forward: segment channels");
            FFC_CHECK_ARG(S.PC > 0 && S.PR > 0, "ffc_convp_forward: patch shape");
            FFC_CHECK_ARG(!S.pool && !S.gate, "ffc_convp_forward: pooled / gated segments use ffc_conv_forward");
            FFC_CHECK_ARG(!S.vec4 || (S.IW % 4 == 0 && S.PC % 4 == 0), "ffc_convp_forward: vec4 staging needs IW, PC % 4 == 0");
            FFC_CHECK_ARG(!S.vec4 || (reinterpret_cast<uintptr_t>(S.x) & 15) == 0,
                          "ffc_convp_forward: vec4 staging needs a 16-byte aligned input");
            const size_t units = (size_t)J.NS * S.cc * S.PR * (S.vec4 ? S.PC / 4 : S.PC);
            FFC_CHECK_ARG(units <= (size_t)NEMAX * 256, "ffc_convp_forward: patch too large for the staging registers");
            const size_t E = (units + 255) / 256 * 256 * (S.vec4 ? 4 : 1);
            if (E > emax) emax = E;
            for (int p = 0; p < J.nphase; ++p) {
                const int T = J.ph[p].T[s];
                FFC_CHECK_ARG(S.cc == 4 ? T == 16 : (T >= 0 && T <= 4 && (T == 0 || (4 % T) == 0)),
                              "ffc_convp_forward: taps must divide 4 (16-channel chunks) or be 16 (4-channel chunks)");
            }
        }
    }
    const size_t ebuf = emax + 64;   // + 64 floats: consecutive buffers start on different banks
    const size_t lds = 2 * ebuf * sizeof(float);
    FFC_CHECK_ARG(lds <= 160 * 1024, "ffc_convp_forward: patch too large");
    ConvPArgs a;
    a.ebuf = (int)ebuf;
    a.jobs[0] = jobs[0];
    a.jobs[1] = jobs[njobs > 1 ? 1 : 0];
    a.tiles = reinterpret_cast<const int4*>(tiles);
    hipStream_t s = (hipStream_t)stream;
    bool pre = true;   // every job carries pre-split A planes
    for (int j = 0; j < njobs; ++j) {
        if (!jobs[j].A3) pre = false;
        FFC_CHECK_ARG(!jobs[j].A3 || (jobs[j].a3_stride % 8 == 0 && (reinterpret_cast<uintptr_t>(jobs[j].A3) & 15) == 0),
                      "ffc_convp_forward: A3 planes need 16-byte alignment");
    }
    if (exact) {
        switch (cfg) {
            case 0: return launch<4, 4, 0>(a, ntiles, lds, s);
            case 1: return launch<4, 2, 0>(a, ntiles, lds, s);
            case 2: return launch<1, 2, 0>(a, ntiles, lds, s);
            case 3: return launch<1, 1, 0>(a, ntiles, lds, s);
        }
    } else if (pre) {
        switch (cfg) {
            case 0: return launch<4, 4, 2>(a, ntiles, lds, s);
            case 1: return launch<4, 2, 2>(a, ntiles, lds, s);
            case 2: return launch<1, 2, 2>(a, ntiles, lds, s);
            case 3: return launch<1, 1, 2>(a, ntiles, lds, s);
        }
    } else {
        switch (cfg) {
            case 0: return launch<4, 4, 1>(a, ntiles, lds, s);
            case 1: return launch<4, 2, 1>(a, ntiles, lds, s);
            case 2: return launch<1, 2, 1>(a, ntiles, lds, s);
            case 3: return launch<1, 1, 1>(a, ntiles, lds, s);
        }
    }
    ffc::set_error("ffc_convp_forward: unknown cfg");
    return FFC_E_INVALID;
}

// ---- ffc_split_bf16: the pre-split packed weights (split3 per element, planes hi / mid / lo)
namespace {
__global__ void split_bf16_kernel(const float* __restrict__ x, long long n, uint16_t* __restrict__ out,
                                  long long stride) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const float a = x[i];
        const unsigned u = __float_as_uint(a);
        const float r1 = a - __uint_as_float(u & 0xFFFF0000u);
        const unsigned u1 = __float_as_uint(r1);
        const float r2 = r1 - __uint_as_float(u1 & 0xFFFF0000u);
        out[i] = (uint16_t)(u >> 16);
        out[stride + i] = (uint16_t)(u1 >> 16);
        out[2 * stride + i] = (uint16_t)(__float_as_uint(r2) >> 16);
    }
}
}  // namespace

extern "C" int ffc_split_bf16(const float* x, long long n, uint16_t* planes, long long stride, void* stream) {
    FFC_CHECK_ARG(x && planes && n > 0 && stride >= n && stride % 8 == 0, "ffc_split_bf16: bad args");
    const long long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(split_bf16_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0,
                       (hipStream_t)stream, x, n, planes, stride);
    return ffc::launch_status("ffc_split_bf16");
}
