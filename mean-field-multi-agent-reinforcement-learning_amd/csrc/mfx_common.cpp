// mfx_common.cpp -- last-error storage and library-level queries of the C ABI.
#include "mfx_common.h"
#include "../../include/magent_amd.h"

#include <hip/hip_runtime.h>

#include <mutex>

namespace mfx {
static std::mutex g_err_mu;
static std::string g_last_error;

void set_last_error(const std::string& msg) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_last_error = msg;
}

int device_cus() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cache[dev]) {
        int n = 0;
        cache[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
    }
    return cache[dev];
}
}  // namespace mfx

extern "C" {

// Last error message of any C-ABI call in this process (empty if none).
MFX_API const char* mfx_last_error() {
    std::lock_guard<std::mutex> lk(mfx::g_err_mu);
    return mfx::g_last_error.c_str();
}

// Library build info; usable without a GPU.
MFX_API const char* mfx_build_info() {
    return "magent_amd: Battle gridworld + Ising MF-Q engine, HIP for gfx950 (CDNA4)";
}

// Number of visible HIP devices (0 without a GPU); never fails.
MFX_API int mfx_device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"
