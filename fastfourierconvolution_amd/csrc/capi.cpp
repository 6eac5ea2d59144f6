// C-ABI plumbing: thread-local error text and launch checks.
#include <hip/hip_runtime.h>

#include <string>

#include "ffc_internal.h"

namespace ffc {

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

int launch_status(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        return FFC_E_LAUNCH;
    }
    return FFC_OK;
}

}  // namespace ffc

extern "C" const char* ffc_last_error(void) { return ffc::g_err.c_str(); }

extern "C" int ffc_abi_version(void) { return 4; }   // 4: ffc_bn_fold.moments, ffc_fu_forward_ex4 (round 6)

// sizes of the ABI structs, so bindings can verify their mirror layouts
extern "C" int ffc_struct_sizes(int* out, int n) {
    if (!out || n < 6) return FFC_E_INVALID;
    out[0] = (int)sizeof(ffc_conv_seg);
    out[1] = (int)sizeof(ffc_conv_phase);
    out[2] = (int)sizeof(ffc_conv_job);
    out[3] = (int)sizeof(ffc_convp_seg);
    out[4] = (int)sizeof(ffc_convp_phase);
    out[5] = (int)sizeof(ffc_convp_job);
    if (n >= 7) out[6] = (int)sizeof(ffc_bn_fold);
    if (n >= 8) out[7] = (int)sizeof(ffc_in_tf);
    if (n >= 10) {
        out[8] = (int)sizeof(ffc_bn_rf_item);
        out[9] = (int)sizeof(ffc_bn_apply_item);
    }
    return FFC_OK;
}
