// LDS-patch implicit-GEMM convolution for gfx950 (f32 MFMA) — the local-branch hot path.
//
// Replaces nn.ConvTranspose2d / nn.Conv2d of FFCTranspose / FFC (layers/ffc/ffc_transpose.py:79-86,
// layers/ffc/ffc.py:45-70) together with SpectralTransform.conv2 (spectral_transform.py:70-71,108),
// which is folded in as a 1x1 segment at the output resolution.
//
// Work decomposition (one workgroup = 4 waves):
//   * 32 output channels (M-tile) x a pixel block (NS samples x TR x TC pixels of the phase grid)
//   * NP = 4 (stride-2 transposed conv): wave w computes phase w = (py, px) of every pixel of the
//     block; NP = 1 (direct conv): the waves split the pixel block.
//   * K runs over (segment, 16-channel chunk, tap).  Per chunk the input patch the block needs is
//     staged once in LDS (zero outside the input, 2x2 avg-pool / SE gate applied on the way in);
//     every (phase, tap) B fragment is a conflict-free ds_read_b32 from it.  The next chunk's
//     global loads are in flight (registers) while the current chunk's MFMAs run.
//   * A (packed weights, k = (seg, ch, tap), each 16-k group of one lane half contiguous) is read
//     straight from L2 as 2 x dwordx4 per lane per 16 k and shared by the wave's N-tiles.
//   * v_mfma_f32_32x32x2_f32: exact fp32.  Lane half h of k-step s carries k = 16g + 8h + s.
#include "ffc_internal.h"

namespace {

constexpr int CC = FFC_PATCH_CC;  // channels per chunk
constexpr int PMAX = 32;          // patch elements staged per thread (patch <= 256 * PMAX floats)

struct ConvPArgs {
    ffc_convp_job jobs[2];
    const int4* tiles;
};

template <int NP, int NTW>
__global__ __launch_bounds__(256) void convp_kernel(ConvPArgs args_byval) {
#if defined(__HIP_DEVICE_COMPILE__)
    const ConvPArgs& args = *(const ConvPArgs*)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const ConvPArgs& args = args_byval;
#endif
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

    const int NS = J.NS, TR = J.TR, TC = J.TC;
    const int bs = pb / (J.nrb * J.ncb);
    const int prem = pb - bs * J.nrb * J.ncb;
    const int rb = prem / J.ncb, cb = prem - rb * J.ncb;
    const int b0 = bs * NS, r0 = rb * TR, c0 = cb * TC;
    const int TRC = TR * TC;

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

    int nchunks = 0;
    for (int s = 0; s < J.nseg; ++s) nchunks += J.seg[s].Cpad / CC;

    float st[PMAX];
    // stage chunk (segment s, channels ch0..ch0+15) into registers
    auto load_chunk = [&](int s, int ch0) {
        const ffc_convp_seg& S = J.seg[s];
        const int PR = S.PR, PC = S.PC;
        const int E = NS * CC * PR * PC;
        const int rpp = 256 / PC;               // rows covered per pass (PC <= 256 checked on host)
        const int col = tid % PC;
        const int rg = tid / PC;
        const bool col_on = rg < rpp;
        // row index R = rg + e*rpp over (ns, ch, pr) rows; track (pr, chn) incrementally
        const int dq = rpp / PR, dr = rpp - (rpp / PR) * PR;
        int pr = rg % PR, chn = rg / PR;
        const int iy0 = r0 * S.mult_y + S.org_y, ix = c0 * S.mult_x + S.org_x + col;
        const bool xin = (unsigned)ix < (unsigned)S.IW;
#pragma unroll
        for (int e = 0; e < PMAX; ++e) {
            float v = 0.0f;
            const int idx = (rg + e * rpp) * PC + col;
            if (col_on && idx < E) {
                const int ns = chn >> 4, ch = chn & 15;
                const int b = b0 + ns, c = ch0 + ch, iy = iy0 + pr;
                if (xin && b < J.B && c < S.C && (unsigned)iy < (unsigned)S.IH) {
                    if (!S.pool) {
                        v = S.x[(((size_t)b * S.C + c) * S.IH + iy) * S.IW + ix];
                    } else {
                        const int W2 = 2 * S.IW;
                        const float* q = S.x + (((size_t)b * S.C + c) * (2 * S.IH) + 2 * iy) * W2 + 2 * ix;
                        v = (((q[0] + q[1]) + q[W2]) + q[W2 + 1]) * 0.25f;
                    }
                    if (S.gate) v *= S.gate[(size_t)b * S.C + c];
                }
            }
            st[e] = v;
            pr += dr;
            chn += dq;
            if (pr >= PR) {
                pr -= PR;
                ++chn;
            }
        }
    };
    auto store_chunk = [&](int s) {
        const ffc_convp_seg& S = J.seg[s];
        const int PC = S.PC;
        const int E = NS * CC * S.PR * PC;
        const int rpp = 256 / PC;
        const int col = tid % PC, rg = tid / PC;
        if (rg < rpp) {
#pragma unroll
            for (int e = 0; e < PMAX; ++e) {
                const int idx = (rg + e * rpp) * PC + col;
                if (idx < E) patch[idx] = st[e];
            }
        }
    };
    auto chunk_seg = [&](int ci, int& s, int& ch0) {
        s = 0;
        while (ci >= J.seg[s].Cpad / CC) {
            ci -= J.seg[s].Cpad / CC;
            ++s;
        }
        ch0 = ci * CC;
    };

    {
        int s, ch0;
        chunk_seg(0, s, ch0);
        load_chunk(s, ch0);
    }
    for (int ci = 0; ci < nchunks; ++ci) {
        int s, ch0;
        chunk_seg(ci, s, ch0);
        __syncthreads();
        store_chunk(s);
        __syncthreads();
        if (ci + 1 < nchunks) {
            int s2, c2;
            chunk_seg(ci + 1, s2, c2);
            load_chunk(s2, c2);
        }
        const int T = P.T[s];
        if (T == 0) continue;
        const ffc_convp_seg& S = J.seg[s];
        const int PRC = S.PR * S.PC;
        int loff[NTW];
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
            loff[nt] = pns[nt] * (CC * PRC) + pr_[nt] * S.mult_y * S.PC + pc_[nt] * S.mult_x;
        const int lt = 31 - __builtin_clz(T);  // T is a power of two dividing 16
        int boff[8];
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) {
            const int k = 8 * h + s8;
            boff[s8] = (k >> lt) * PRC + J.taptab[P.tap_base[s] + (k & (T - 1))];
        }
        const int gstep = (16 >> lt) * PRC;
        const float* __restrict__ Ap = J.A + P.a_off + (size_t)(m0 + cl) * P.Kpad + P.kseg[s] + ch0 * T + 8 * h;
        float4 a0 = *reinterpret_cast<const float4*>(Ap);
        float4 a1 = *reinterpret_cast<const float4*>(Ap + 4);
        for (int g = 0; g < T; ++g) {
            float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            if (g + 1 < T) {
                a0 = *reinterpret_cast<const float4*>(Ap + 16 * (g + 1));
                a1 = *reinterpret_cast<const float4*>(Ap + 16 * (g + 1) + 4);
            }
            const int go = g * gstep;
#pragma unroll
            for (int s8 = 0; s8 < 8; ++s8) {
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt) {
                    const float bv = patch[loff[nt] + boff[s8] + go];
                    acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s8], bv, acc[nt], 0, 0, 0);
                }
            }
        }
    }

    // ---------------- epilogue: bias/addend, BN partials, activation, store
    const size_t plane = (size_t)J.OH * J.OW;
    int ob[NTW], oo[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
        ob[nt] = b0 + pns[nt];
        oo[nt] = ((r0 + pr_[nt]) * J.Sy + P.py) * J.OW + ((c0 + pc_[nt]) * J.Sx + P.px);
    }
    const int mbase = m0 + 4 * h;
    if (J.bias || J.addend) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + (r & 3) + 8 * (r >> 2);
            if (m >= J.M) continue;
            const float bv = J.bias ? J.bias[m] : 0.0f;
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
                float v = acc[nt][r] + bv;
                if (J.addend && pv[nt]) v += J.addend[((size_t)ob[nt] * J.M + m) * plane + oo[nt]];
                acc[nt][r] = v;
            }
        }
    }
    if (J.stats) {
        float cntl = 0.0f;
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) cntl += pv[nt] ? 1.0f : 0.0f;
        const float cnt = ffc::half_wave_sum(cntl);
        float4* stp = reinterpret_cast<float4*>(J.stats) + ((size_t)pb * 4 + wave) * J.M;
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
            if (cl == 0 && m < J.M) stp[m] = make_float4(cnt, mean, m2, 0.0f);
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = mbase + (r & 3) + 8 * (r >> 2);
        if (m >= J.M) continue;
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
            if (pv[nt])
                J.out[((size_t)ob[nt] * J.M + m) * plane + oo[nt]] = ffc::apply_act(acc[nt][r], J.act, J.act_param);
    }
}

template <int NP, int NTW>
int launch(const ConvPArgs& a, int ntiles, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((convp_kernel<NP, NTW>), dim3(ntiles), dim3(256), lds, s, a);
    return ffc::launch_status("ffc_convp_forward");
}

}  // namespace

extern "C" int ffc_convp_forward(const ffc_convp_job* jobs, int njobs, const int* tiles, int ntiles, int cfg,
                                 void* stream) {
    FFC_CHECK_ARG(jobs && tiles && njobs >= 1 && njobs <= 2 && ntiles > 0, "ffc_convp_forward: bad args");
    size_t emax = 0;
    const int np = (cfg <= 1) ? 4 : 1;
    for (int j = 0; j < njobs; ++j) {
        const ffc_convp_job& J = jobs[j];
        FFC_CHECK_ARG(J.A && J.taptab && J.out && J.B > 0 && J.M > 0, "ffc_convp_forward: incomplete job");
        FFC_CHECK_ARG(J.nphase == np, "ffc_convp_forward: phase count does not match cfg");
        FFC_CHECK_ARG(J.nseg >= 1 && J.nseg <= FFC_MAX_SEG, "ffc_convp_forward: nseg out of range");
        FFC_CHECK_ARG(J.Mpad % 128 == 0 && J.Mpad >= J.M, "ffc_convp_forward: Mpad");
        FFC_CHECK_ARG(J.NS > 0 && J.TR > 0 && J.TC > 0 && J.nrb > 0 && J.ncb > 0, "ffc_convp_forward: tiling");
        for (int s = 0; s < J.nseg; ++s) {
            const ffc_convp_seg& S = J.seg[s];
            FFC_CHECK_ARG(S.x && S.Cpad % CC == 0 && S.Cpad >= S.C, "ffc_convp_forward: segment channels");
            FFC_CHECK_ARG(S.PC > 0 && S.PC <= 256 && S.PR > 0, "ffc_convp_forward: patch shape");
            const size_t E = (size_t)J.NS * CC * S.PR * S.PC;
            const size_t rows = (size_t)J.NS * CC * S.PR;
            FFC_CHECK_ARG(rows <= (size_t)(256 / S.PC) * PMAX, "ffc_convp_forward: patch exceeds staging registers");
            if (E > emax) emax = E;
            for (int p = 0; p < J.nphase; ++p) {
                const int T = J.ph[p].T[s];
                FFC_CHECK_ARG(T >= 0 && T <= 16 && (T == 0 || (16 % T) == 0), "ffc_convp_forward: taps must divide 16");
            }
        }
    }
    const size_t lds = emax * sizeof(float);
    FFC_CHECK_ARG(lds <= 64 * 1024, "ffc_convp_forward: patch too large");
    ConvPArgs a;
    a.jobs[0] = jobs[0];
    a.jobs[1] = jobs[njobs > 1 ? 1 : 0];
    a.tiles = reinterpret_cast<const int4*>(tiles);
    hipStream_t s = (hipStream_t)stream;
    switch (cfg) {
        case 0: return launch<4, 4>(a, ntiles, lds, s);
        case 1: return launch<4, 2>(a, ntiles, lds, s);
        case 2: return launch<1, 2>(a, ntiles, lds, s);
        case 3: return launch<1, 1>(a, ntiles, lds, s);
    }
    ffc::set_error("ffc_convp_forward: unknown cfg");
    return FFC_E_INVALID;
}
