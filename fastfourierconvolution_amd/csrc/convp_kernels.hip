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

#include <string>

namespace {

constexpr int CC = FFC_PATCH_CC;  // channels per chunk

struct ConvPArgs {
    ffc_convp_job jobs[2];
    const int4* tiles;
    int ebuf;                      // floats per LDS patch buffer (multiple of 256)
};

__device__ float g_zero_src[64];   // source of the zero fill for out-of-bounds patch elements

typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

__device__ __forceinline__ unsigned magic_div(unsigned d) { return 0xFFFFFFFFu / d + 1u; }

// Stage one 16-channel chunk of segment S into LDS `dst` with LDS-DMA (global_load_lds_dword):
// element n of the patch image [ns][ch][pr][pc] comes from lane n % 64 of wave-instruction n / 64;
// out-of-range elements read a zero word.  No VGPR staging, no branches.
__device__ __forceinline__ void stage_chunk(const ffc_convp_seg& S, int NS, int B, int b0, int r0, int c0,
                                            int ch0, float* dst, int tid, int wave) {
    const int PR = S.PR, PC = S.PC;
    const int E = NS * CC * PR * PC;
    const unsigned mPC = magic_div((unsigned)PC), mPR = magic_div((unsigned)PR);
    const int iy0 = r0 * S.mult_y + S.org_y, ix0 = c0 * S.mult_x + S.org_x;
    const int nE = (E + 255) >> 8;
    for (int e = 0; e < nE; ++e) {
        const unsigned n = (unsigned)(e * 256 + tid);
        const unsigned q1 = __umulhi(n, mPC);
        const int pc = (int)(n - q1 * PC);
        const unsigned q2 = __umulhi(q1, mPR);
        const int pr = (int)(q1 - q2 * PR);
        const int ns = (int)(q2 >> 4), ch = (int)(q2 & 15);
        const int b = b0 + ns, c = ch0 + ch, iy = iy0 + pr, ix = ix0 + pc;
        const bool ok = (int)n < E && b < B && c < S.C && (unsigned)iy < (unsigned)S.IH &&
                        (unsigned)ix < (unsigned)S.IW;
        const float* src = ok ? S.x + (unsigned)(((b * S.C + c) * S.IH + iy) * S.IW + ix) : g_zero_src;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + e * 256 + wave * 64), 4, 0, 0);
    }
}

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
    const int ebuf = args.ebuf;

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
    auto chunk_seg = [&](int ci, int& s, int& ch0) {
        s = 0;
        while (ci >= J.seg[s].Cpad / CC) {
            ci -= J.seg[s].Cpad / CC;
            ++s;
        }
        ch0 = ci * CC;
    };
    // A (16-k groups, T <= 4 per chunk) of chunk ci into registers (not waited for here)
    auto load_A = [&](int ci, floatx4 (&a0)[4], floatx4 (&a1)[4]) {
        int s, ch0;
        chunk_seg(ci, s, ch0);
        const int T = P.T[s];
        const float* __restrict__ Ap = J.A + P.a_off + (size_t)(m0 + cl) * P.Kpad + P.kseg[s] + ch0 * T + 8 * h;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (g < T) {
                a0[g] = *reinterpret_cast<const floatx4*>(Ap + 16 * g);
                a1[g] = *reinterpret_cast<const floatx4*>(Ap + 16 * g + 4);
            } else {
                a0[g] = floatx4{0.f, 0.f, 0.f, 0.f};
                a1[g] = a0[g];
            }
        }
    };
    auto stage = [&](int ci) {
        int s, ch0;
        chunk_seg(ci, s, ch0);
        stage_chunk(J.seg[s], NS, J.B, b0, r0, c0, ch0, patch + (ci & 1) * ebuf, tid, wave);
    };
    floatx4 a0[4], a1[4], n0[4], n1[4];
    stage(0);
    load_A(0, n0, n1);
    for (int ci = 0; ci < nchunks; ++ci) {
        int s, ch0;
        chunk_seg(ci, s, ch0);
        __syncthreads();  // patch + A of chunk ci landed (vmcnt(0)); everyone is done with chunk ci-1
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            a0[g] = n0[g];
            a1[g] = n1[g];
            asm volatile("" : "+v"(a0[g]), "+v"(a1[g]));
        }
        if (ci + 1 < nchunks) {  // next chunk's A and patch stay in flight under this chunk's MFMAs
            load_A(ci + 1, n0, n1);
            stage(ci + 1);
        }
        const int T = P.T[s];
        if (T == 0) continue;
        const ffc_convp_seg& S = J.seg[s];
        const int lt = 31 - __builtin_clz(T);  // T is a power of two dividing 4
        const float* cur = patch + (ci & 1) * ebuf;
        const int PRC = S.PR * S.PC;
        int loff[NTW];
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
            loff[nt] = pns[nt] * (CC * PRC) + pr_[nt] * S.mult_y * S.PC + pc_[nt] * S.mult_x;
        int boff[8];
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) {
            const int k = 8 * h + s8;
            boff[s8] = (k >> lt) * PRC + J.taptab[P.tap_base[s] + (k & (T - 1))];
        }
        const int gstep = (16 >> lt) * PRC;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (g < T) {
                const float av[8] = {a0[g][0], a0[g][1], a0[g][2], a0[g][3], a1[g][0], a1[g][1], a1[g][2], a1[g][3]};
                int go = g * gstep;
                asm volatile("" : "+s"(go));  // keep the per-group LDS addresses from being hoisted (VGPRs)
                const float* cg = cur + go;
#pragma unroll
                for (int s8 = 0; s8 < 8; ++s8) {
#pragma unroll
                    for (int nt = 0; nt < NTW; ++nt) {
                        const float bv = cg[loff[nt] + boff[s8]];
                        acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s8], bv, acc[nt], 0, 0, 0);
                    }
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
    auto store = [&](auto actf) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + (r & 3) + 8 * (r >> 2);
            if (m < J.M) {
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt)
                    if (pv[nt]) J.out[((size_t)ob[nt] * J.M + m) * plane + oo[nt]] = actf(acc[nt][r]);
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
}

template <int NP, int NTW>
int launch(const ConvPArgs& a, int ntiles, size_t lds, hipStream_t s) {
    auto k = convp_kernel<NP, NTW>;
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
            FFC_CHECK_ARG(S.PC > 0 && S.PR > 0, "ffc_convp_forward: patch shape");
            FFC_CHECK_ARG(!S.pool && !S.gate, "ffc_convp_forward: pooled / gated segments use ffc_conv_forward");
            const size_t E = (size_t)J.NS * CC * S.PR * S.PC;
            if (E > emax) emax = E;
            for (int p = 0; p < J.nphase; ++p) {
                const int T = J.ph[p].T[s];
                FFC_CHECK_ARG(T >= 0 && T <= 4 && (T == 0 || (4 % T) == 0), "ffc_convp_forward: taps must divide 4");
            }
        }
    }
    const size_t ebuf = (emax + 255) / 256 * 256 + 256;
    const size_t lds = 2 * ebuf * sizeof(float);
    FFC_CHECK_ARG(lds <= 160 * 1024, "ffc_convp_forward: patch too large");
    ConvPArgs a;
    a.ebuf = (int)ebuf;
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
