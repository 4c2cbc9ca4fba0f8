// mfx_common.h -- error plumbing and small device-buffer helper shared by the host runtimes.
//
// Error convention of the C ABI: 0 = success; -1 = failure, with the message printed to
// stderr and retrievable through mfx_last_error().  (The reference returns 0 and aborts on
// LOG(FATAL); this library reports instead of aborting, and the drop-in python raises.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <stdexcept>
#include <string>

#define MFX_API __attribute__((visibility("default")))

namespace mfx {

void set_last_error(const std::string& msg);

// Compute units of the current device (256 on MI355X; 256 when the query fails), per device, cached.
int device_cus();

inline int fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
inline int fail(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    fprintf(stderr, "[magent_amd] %s\n", buf);
    set_last_error(buf);
    return -1;
}

struct HipFailure : std::runtime_error {
    using std::runtime_error::runtime_error;
};

}  // namespace mfx

#define MFX_HIP(expr)                                                                    \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
            return mfx::fail("HIP error %s at %s:%d", hipGetErrorString(_e), __FILE__, __LINE__); \
    } while (0)

#define MFX_HIP_THROW(expr)                                                              \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
            throw mfx::HipFailure(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                                  __FILE__ + ":" + std::to_string(__LINE__));            \
    } while (0)

#define MFX_CHECK(expr)            \
    do {                           \
        int _r = (expr);           \
        if (_r != 0) return _r;    \
    } while (0)

namespace mfx {

template <class T>
struct PinBuf {                    // grow-only pinned host buffer (async DMA target / source)
    T* p = nullptr;
    size_t n = 0;
    void ensure(size_t want) {
        if (want <= n) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        MFX_HIP_THROW(hipHostMalloc((void**)&p, sizeof(T) * want, hipHostMallocDefault));
        n = want;
    }
    ~PinBuf() { if (p) (void)hipHostFree(p); }
};

template <class T>
struct MappedBuf {                 // grow-only pinned host buffer the device reads / writes in place
    T* p = nullptr;                //   host address
    T* d = nullptr;                //   the device's address of the same memory
    size_t n = 0;
    void ensure(size_t want, unsigned flags = 0) {
        if (want <= n) return;
        if (p) (void)hipHostFree(p);
        p = d = nullptr;
        MFX_HIP_THROW(hipHostMalloc((void**)&p, sizeof(T) * want, hipHostMallocMapped | flags));
        MFX_HIP_THROW(hipHostGetDevicePointer((void**)&d, p, 0));
        n = want;
    }
    ~MappedBuf() { if (p) (void)hipHostFree(p); }
};

template <class T>
struct DevBuf {                    // grow-only device buffer
    T* p = nullptr;
    size_t n = 0;
    void ensure(size_t want) {
        if (want <= n) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        MFX_HIP_THROW(hipMalloc(&p, sizeof(T) * want));
        n = want;
    }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

}  // namespace mfx
