// Host-side sanitizer driver for the C ABI (SURVEY.md §5 "race detection / sanitizers").
//
// Linked against a host-only build of every csrc/ source (hipcc --cuda-host-only, no device code)
// instrumented with AddressSanitizer + UndefinedBehaviorSanitizer, or with ThreadSanitizer
// (tests/test_sanitizers_cpu.py builds both).  No GPU is touched: every call below is rejected by
// the entry point's argument validation before any HIP call, so the run exercises exactly the
// host code a binding reaches first -- the validation, the shape queries' size arithmetic and the
// thread-local error text (ffc_last_error) -- under the sanitizers.
//
//   ./abi_sanitize            exit 0 and "abi_sanitize: N checks ok" on success
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ffc_amd.h"

static int g_checks = 0, g_fail = 0;

#define EXPECT_INVALID(call, needle)                                                              \
    do {                                                                                          \
        const int rc_ = (call);                                                                   \
        ++g_checks;                                                                               \
        const char* e_ = ffc_last_error();                                                        \
        if (rc_ != FFC_E_INVALID || !e_ || !std::strstr(e_, needle)) {                            \
            std::fprintf(stderr, "FAIL %s:%d %s -> %d '%s'\n", __FILE__, __LINE__, #call, rc_,     \
                         e_ ? e_ : "(null)");                                                     \
            ++g_fail;                                                                             \
        }                                                                                         \
    } while (0)

#define EXPECT_EQ(a, b)                                                                           \
    do {                                                                                          \
        ++g_checks;                                                                               \
        if (!((a) == (b))) {                                                                      \
            std::fprintf(stderr, "FAIL %s:%d %s != %s\n", __FILE__, __LINE__, #a, #b);            \
            ++g_fail;                                                                             \
        }                                                                                         \
    } while (0)

alignas(16) static float buf[4096];
alignas(16) static double dbuf[64];

static void validation_paths() {
    float* p = buf;
    const float* cp = buf;
    // --- batch norm / SE / caller ops (bn_se_kernels.hip, caller_kernels.hip)
    EXPECT_INVALID(ffc_bn_reduce(nullptr, 4, 4, dbuf, nullptr), "ffc_bn_reduce");
    EXPECT_INVALID(ffc_bn_reduce(cp, 0, 4, dbuf, nullptr), "ffc_bn_reduce");
    EXPECT_INVALID(ffc_bn_finalize(dbuf, 0, cp, cp, p, p, nullptr, 1, 0, 0.1f, 1e-5f, 1.f, p, p, nullptr),
                   "ffc_bn_finalize");
    EXPECT_INVALID(ffc_bn_finalize(nullptr, 4, cp, cp, p, p, nullptr, 1, 0, 0.1f, 1e-5f, 1.f, p, p, nullptr),
                   "batch stats need moments");
    EXPECT_INVALID(ffc_bn_finalize(dbuf, 4, cp, cp, nullptr, p, nullptr, 0, 0, 0.1f, 1e-5f, 1.f, p, p, nullptr),
                   "eval needs running stats");
    EXPECT_INVALID(ffc_bn_finalize(dbuf, 4, cp, cp, p, p, nullptr, 1, 1, 0.1f, 1e-5f, 1.f, p, p, nullptr),
                   "update needs running buffers");
    EXPECT_INVALID(ffc_bn_reduce_finalize(cp, 4, 4, dbuf, cp, cp, p, p, nullptr, 1, 0.1f, 1e-5f, 1.f, p, p, nullptr),
                   "update needs running buffers");
    EXPECT_INVALID(ffc_bn_reduce_finalize(cp, 4, 4, dbuf, cp, cp, p, p, nullptr, 0, 0.1f, 1e-5f, 1.f, nullptr, p,
                                          nullptr), "ffc_bn_reduce_finalize");
    EXPECT_INVALID(ffc_bn_act_apply(cp, p, 0, 4, 16, cp, cp, 0, 0.f, nullptr), "ffc_bn_act_apply");
    EXPECT_INVALID(ffc_bn_act_noise_apply(cp, p, 1, 4, 6, cp, cp, 0, 0.f, cp, cp, nullptr), "ffc_bn_act_noise_apply");
    EXPECT_INVALID(ffc_bn_act_noise_apply(cp, p, 1, 4, 8, cp, cp, 0, 0.f, nullptr, cp, nullptr), "ffc_bn_act_noise_apply");
    EXPECT_INVALID(ffc_se_gate(cp, 1, 4, 4, 4, 0, nullptr, nullptr, 2, p, nullptr), "null weights");
    EXPECT_INVALID(ffc_se_gate(cp, 1, 4, 4, 4, 0, nullptr, nullptr, -1, p, nullptr), "ffc_se_gate");
    EXPECT_INVALID(ffc_noise_inject(cp, cp, cp, p, 1, 4, 6, nullptr), "multiple of 4");
    EXPECT_INVALID(ffc_noise_inject(cp, nullptr, cp, p, 1, 4, 8, nullptr), "null pointer");
    EXPECT_INVALID(ffc_noise_wgrad(cp, cp, 1, 4, 6, p, nullptr), "multiple of 4");
    EXPECT_INVALID(ffc_noise_wgrad(nullptr, cp, 1, 4, 8, p, nullptr), "null pointer");
    if (ffc_bn_reduce_ws_doubles(100, 64) != 0 || ffc_bn_reduce_ws_doubles(0, 64) != 0 ||
        ffc_bn_reduce_ws_doubles(1 << 30, 1 << 12) == 0) {
        std::fprintf(stderr, "FAIL ffc_bn_reduce_ws_doubles\n");
        ++g_fail;
    }
    EXPECT_INVALID(ffc_quantize_u8(cp, reinterpret_cast<unsigned char*>(p), 6, nullptr), "ffc_quantize_u8");
    // --- convolution jobs (conv_kernels.hip, convp_kernels.hip, pw_gemm.hip, dense.hip, convt_smallm.hip)
    ffc_conv_job job;
    std::memset(&job, 0, sizeof(job));
    int tiles[4] = {0, 0, 0, 0};
    EXPECT_INVALID(ffc_conv_forward(nullptr, 1, tiles, 1, 0, nullptr), "ffc_conv_forward");
    EXPECT_INVALID(ffc_conv_forward(&job, 3, tiles, 1, 0, nullptr), "ffc_conv_forward");
    EXPECT_INVALID(ffc_conv_forward(&job, 1, tiles, 1, 0, nullptr), "incomplete job");
    job.A = cp;
    job.ktab = tiles;
    job.out = p;
    job.B = job.M = 1;
    job.nseg = 4;
    EXPECT_INVALID(ffc_conv_forward(&job, 1, tiles, 1, 0, nullptr), "nseg out of range");
    job.nseg = 1;
    job.nphase = 1;
    job.Mpad = 100;
    EXPECT_INVALID(ffc_conv_forward(&job, 1, tiles, 1, 0, nullptr), "Mpad");
    job.Mpad = 128;
    job.ph[0].K = 16;
    job.ph[0].Kpad = 16;
    EXPECT_INVALID(ffc_conv_forward(&job, 1, tiles, 1, 0, nullptr), "null segment");
    EXPECT_INVALID(ffc_conv_pack(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, p, p, nullptr), "ffc_conv_pack");
    EXPECT_INVALID(ffc_pw_forward(&job, 5, nullptr), "ffc_pw_forward");
    job.stats = p;
    job.ph[0].a_off = 0;
    EXPECT_INVALID(ffc_pw_forward(&job, 0, nullptr), "BN partials");
    ffc_convp_job pj;
    std::memset(&pj, 0, sizeof(pj));
    EXPECT_INVALID(ffc_convp_forward(&pj, 0, tiles, 1, 0, nullptr), "ffc_convp_forward");
    EXPECT_INVALID(ffc_convp_forward(&pj, 1, tiles, 1, 0, nullptr), "incomplete job");
    EXPECT_INVALID(ffc_split_bf16(cp, 16, reinterpret_cast<uint16_t*>(p), 12, nullptr), "ffc_split_bf16");
    EXPECT_INVALID(ffc_convq_forward(&pj, 0, tiles, 1, 0, nullptr), "ffc_convq_forward");
    EXPECT_INVALID(ffc_convq_forward(&pj, 1, tiles, 1, 7, nullptr), "unknown cfg");
    EXPECT_INVALID(ffc_convq_forward(&pj, 1, tiles, 1, 0, nullptr), "needs the A3 planes");
    EXPECT_INVALID(ffc_convq_forward_split(&pj, 1, tiles, 1, tiles, 1, 0, 9, p, nullptr), "ksplit <= 8");
    EXPECT_INVALID(ffc_convq_forward_split(&pj, 1, tiles, 2, tiles, 1, 0, 2, nullptr, nullptr), "partial buffer");
    EXPECT_INVALID(ffc_convq_forward_split(&pj, 1, tiles, 3, tiles, 1, 0, 2, p, nullptr), "slot table");
    EXPECT_INVALID(ffc_convq_pack_a3(nullptr, cp, reinterpret_cast<uint16_t*>(p), nullptr), "ffc_convq_pack_a3");
    EXPECT_INVALID(ffc_dense_forward(cp, cp, nullptr, 1, 300, 8, 8, p, nullptr, 0, 0.f, nullptr), "K > 256");
    EXPECT_INVALID(ffc_dense_forward(cp, cp, nullptr, 1, 16, 8, 4, p, nullptr, 0, 0.f, nullptr), "output split");
    EXPECT_INVALID(ffc_convt_smallm_pack(cp, 4, nullptr, 0, 5, p, nullptr), "");
    EXPECT_INVALID(ffc_convt_k4s2_smallm(cp, 4, nullptr, 0, cp, nullptr, 1, 4, 4, 5, p, 0, 0.f, nullptr), "M <= 4");
    EXPECT_INVALID(ffc_convt_k4s2_smallm(cp, 300, nullptr, 0, cp, nullptr, 1, 4, 4, 3, p, 0, 0.f, nullptr),
                   "256 input channels");
    EXPECT_INVALID(ffc_conv3x3_smallm(cp, 4, cp, cp, 4, nullptr, nullptr, 1, 8, 8, 3, p, 0, 0.f, nullptr),
                   "second segment");
    EXPECT_INVALID(ffc_conv3x3_smallm(cp, 4, cp, nullptr, 0, nullptr, nullptr, 1, 8, 6, 3, p, 0, 0.f, nullptr),
                   "ffc_conv3x3_smallm");
    {
        const ffc_in_tf bad = {nullptr, nullptr, 0, 0.f, nullptr, nullptr};
        EXPECT_INVALID(ffc_conv3x3_smallm_tf(cp, 4, cp, nullptr, 0, nullptr, nullptr, 1, 8, 8, 3, p, 0, 0.f, &bad,
                                             nullptr, nullptr), "scale");
        EXPECT_INVALID(ffc_fu2d_c2r_bn(cp, 1, 4, 32, 32, cp, 2, nullptr, nullptr, 0, 1, nullptr, nullptr, p, nullptr),
                       "bn_scale");
    }
    // --- spectral branch (st_prologue.hip, st_pw.hip, fu_kernels.hip, fu2d_kernels.hip)
    EXPECT_INVALID(ffc_st_prologue(cp, 1, 4096, 64, 64, 0, nullptr, nullptr, 0, cp, 4, p, p, nullptr, nullptr),
                   "does not fit");
    EXPECT_INVALID(ffc_st_prologue(cp, 1, 16, 8, 8, 0, nullptr, nullptr, 1, cp, 4, p, p, nullptr, nullptr),
                   "null SE weights");
    EXPECT_INVALID(ffc_pw_gate_conv(cp, nullptr, cp, 1, 16, 1000, 64, p, nullptr, nullptr), "unsupported");
    EXPECT_INVALID(ffc_pack_transpose(cp, 0, 4, p, nullptr), "ffc_pack_transpose");
    EXPECT_INVALID(ffc_fu_forward(cp, 1, 4, 12, 12, 1, nullptr, nullptr, 0, cp, 0, p, nullptr, nullptr, 0, nullptr,
                                  nullptr), "unsupported");
    EXPECT_INVALID(ffc_fu_forward(cp, 1, 4, 8, 8, 3, nullptr, nullptr, 0, cp, 0, p, nullptr, nullptr, 0, nullptr,
                                  nullptr), "up must be");
    EXPECT_INVALID(ffc_fu_forward(cp, 1, 4, 8, 8, 1, cp, nullptr, 0, cp, 0, p, nullptr, nullptr, 0, nullptr, nullptr),
                   "pairing");
    EXPECT_INVALID(ffc_fu_forward(cp, 1, 4, 8, 8, 1, nullptr, nullptr, 0, cp, 1, nullptr, nullptr, nullptr, 0,
                                  nullptr, nullptr), "pass 1 needs");
    {
        ffc_bn_fold f;
        std::memset(&f, 0, sizeof(f));
        f.slab = cp;
        f.nrows = 1;
        f.C = 4;
        EXPECT_INVALID(ffc_fu_forward_ex(cp, 1, 4, 8, 8, 1, nullptr, nullptr, 1, cp, 0, p, nullptr, nullptr, 0, nullptr,
                                         &f, nullptr, nullptr, nullptr), "needs scale_out");
        f.scale_out = p;
        f.shift_out = p;
        f.update_running = 1;
        EXPECT_INVALID(ffc_fu_forward_ex(cp, 1, 4, 8, 8, 1, nullptr, nullptr, 1, cp, 0, p, nullptr, nullptr, 0, nullptr,
                                         &f, nullptr, nullptr, nullptr), "incomplete ffc_bn_fold");
        f.update_running = 0;
        EXPECT_INVALID(ffc_fu_forward_ex(cp, 1, 4, 8, 8, 1, nullptr, nullptr, 1, cp, 0, p, nullptr, nullptr, 0, nullptr,
                                         nullptr, &f, nullptr, nullptr), "mix_fold is pass 1 only");
        EXPECT_INVALID(ffc_fu_forward_ex(cp, 1, 4, 8, 8, 1, nullptr, nullptr, 1, cp, 1, nullptr, nullptr, nullptr, 0, p,
                                         nullptr, &f, nullptr, nullptr), "mix_fold->C != 2C");
    }
    EXPECT_INVALID(ffc_fu2d_r2c(cp, 1, 4, 48, 48, nullptr, nullptr, 0, p, nullptr), "unsupported plane");
    EXPECT_INVALID(ffc_fu2d_mix(cp, 1, 65, 64, 64, 1, cp, 0, p, nullptr, nullptr, nullptr, nullptr), "unsupported");
    EXPECT_INVALID(ffc_fu2d_mix(cp, 1, 8, 64, 64, 1, cp, 2, p, nullptr, nullptr, nullptr, nullptr), "pass must be");
    EXPECT_INVALID(ffc_fu2d_mix_f16(cp, 1, 8, 64, 64, 1, cp, 0, p, nullptr, nullptr, nullptr, nullptr), "C must be");
    EXPECT_INVALID(ffc_fu_pack_mix_f16(cp, 0, p, nullptr), "ffc_fu_pack_mix_f16");
    EXPECT_INVALID(ffc_fu2d_c2r(cp, 1, 4, 64, 64, nullptr, 1, nullptr, nullptr, 0, 1, p, nullptr), "residual needs t");
    EXPECT_INVALID(ffc_fu2d_c2r(cp, 1, 4, 64, 64, cp, 3, nullptr, nullptr, 0, 1, p, nullptr), "up must be");
    EXPECT_INVALID(ffc_fu2d_mix_cols(cp, 1, 4, 64, 48, 1, cp, 0, cp, cp, p, nullptr), "unsupported");
    EXPECT_INVALID(ffc_fu2d_c2r_rows(cp, 1, 4, 16, 16, cp, 1, nullptr, nullptr, 0, 0, p, nullptr), "unsupported plane");
    // --- training path (train_kernels.hip)
    EXPECT_INVALID(ffc_act_bwd(cp, cp, p, 16, 9, 0.f, nullptr), "ffc_act_bwd");
    EXPECT_INVALID(ffc_bn_bwd_sums(cp, cp, 1, 4, 16, cp, cp, 0, 0.f, dbuf, 0, dbuf, nullptr), "ffc_bn_bwd_sums");
    EXPECT_INVALID(ffc_bn_bwd_coeff(dbuf, 4, nullptr, 1e-5f, nullptr, p, nullptr, nullptr, nullptr), "ffc_bn_bwd_coeff");
    EXPECT_INVALID(ffc_bn_bwd_apply(cp, cp, 1, 4, 16, cp, cp, 0, 0.f, cp, nullptr, nullptr), "ffc_bn_bwd_apply");
    EXPECT_INVALID(ffc_channel_moments(cp, 1, 4, 16, dbuf, 0, dbuf, nullptr), "ffc_channel_moments");
    EXPECT_INVALID(ffc_bn_bwd(cp, cp, 1, 4, 16, cp, cp, 0, 0.f, nullptr, nullptr, nullptr, 1e-5f, cp, dbuf, 1, p,
                              nullptr, nullptr, p, nullptr), "need batch moments");
    EXPECT_INVALID(ffc_conv_wgrad(cp, 4, 4, 4, cp, 4, 4, 4, 1, 3, 1, 1, 1, 2, nullptr, p, 0, nullptr), "workspace");
    EXPECT_INVALID(ffc_rfft2_planes(cp, 1, 128, 96, 1.f, p, nullptr), "ffc_rfft2_planes");
    EXPECT_INVALID(ffc_irfft2_planes(cp, 1, 8, 1, 1.f, nullptr, p, nullptr), "ffc_irfft2_planes");
    EXPECT_INVALID(ffc_se_bwd(cp, cp, 1, 4, 4, 4, nullptr, nullptr, 40, p, p, p, p, p, p, nullptr), "ffc_se_bwd");
    EXPECT_INVALID(ffc_conv_full_smallm(cp, 16, cp, nullptr, 0, nullptr, nullptr, 1, 9, p, 0, 0.f, nullptr),
                   "ffc_conv_full_smallm");
    EXPECT_INVALID(ffc_pool2(cp, 1, 3, 4, 0.25f, p, nullptr), "ffc_pool2");
    EXPECT_INVALID(ffc_up2(cp, 0, 4, 4, 1.f, p, nullptr), "ffc_up2");
}

static void shape_queries() {
    // size arithmetic over extreme arguments must not overflow (UBSan) or read out of bounds (ASan)
    const int vals[] = {-1, 0, 1, 2, 3, 4, 7, 8, 16, 32, 64, 96, 128, 256, 4096, 1 << 20, 0x7fffffff};
    for (int a : vals)
        for (int b : vals) {
            (void)ffc_fu_lds_bytes(a, b, b);
            (void)ffc_fu2d_supported(a, b, b, 1);
            (void)ffc_fu2d_supported(a, b, b, 2);
            (void)ffc_fu2d_cols_supported(a, b, b, 1, 0);
            (void)ffc_fu2d_cols_supported(a, b, b, 2, 1);
            (void)ffc_st_prologue_lds_bytes(a, b, b, 0, a / 16, b);
            (void)ffc_pw_gate_lds_bytes(a, b);
            (void)ffc_pw_gate_blocks(b);
            (void)ffc_convt_smallm_pack_floats(a, b);
            (void)ffc_conv_stat_rows_per_tile(a & 3);
        }
    for (int cfg = -1; cfg < 6; ++cfg)
        for (int ks = -1; ks < 10; ++ks) (void)ffc_convq_split_floats(cfg, 1 << 20, ks);
    int mt = 0, ntw = 0;
    EXPECT_EQ(ffc_convq_config(2, &mt, &ntw), FFC_OK);
    EXPECT_EQ(mt * 10 + ntw, 22);
    EXPECT_EQ(ffc_convq_config(4, &mt, &ntw), FFC_E_INVALID);
    EXPECT_EQ(ffc_convq_split_floats(3, 10, 4), 10LL * 4 * 4 * 1024);
    EXPECT_EQ(ffc_convq_split_floats(0, 10, 1), 0LL);
    EXPECT_EQ(ffc_convq_split_floats(0, 10, 9), -1LL);
    EXPECT_EQ(ffc_fu_lds_bytes(16, 64, 64), (size_t)0);
    EXPECT_EQ(ffc_fu2d_supported(65, 64, 64, 1), 0);
    EXPECT_EQ(ffc_fu2d_supported(32, 128, 128, 1), 1);
    int sizes[6];
    EXPECT_EQ(ffc_struct_sizes(sizes, 6), FFC_OK);
    EXPECT_EQ(ffc_struct_sizes(sizes, 5), FFC_E_INVALID);
    EXPECT_EQ(ffc_abi_version(), 4);
}

// ffc_last_error is thread-local: concurrent failing calls each see their own message
static void threaded_errors() {
    std::atomic<int> bad{0};
    std::vector<std::thread> ts;
    for (int i = 0; i < 8; ++i)
        ts.emplace_back([i, &bad] {
            for (int r = 0; r < 2000; ++r) {
                int rc;
                const char* want;
                if ((i + r) % 2) {
                    rc = ffc_up2(buf, 0, 4, 4, 1.f, buf, nullptr);
                    want = "ffc_up2";
                } else {
                    rc = ffc_pool2(buf, 1, 3, 4, 0.25f, buf, nullptr);
                    want = "ffc_pool2";
                }
                const std::string e = ffc_last_error();
                if (rc != FFC_E_INVALID || e.find(want) == std::string::npos) ++bad;
            }
        });
    for (auto& t : ts) t.join();
    ++g_checks;
    if (bad) {
        std::fprintf(stderr, "FAIL threaded_errors: %d mismatched messages\n", bad.load());
        ++g_fail;
    }
}

int main() {
    validation_paths();
    shape_queries();
    threaded_errors();
    if (g_fail) {
        std::fprintf(stderr, "abi_sanitize: %d of %d checks failed\n", g_fail, g_checks);
        return 1;
    }
    std::printf("abi_sanitize: %d checks ok\n", g_checks);
    return 0;
}
