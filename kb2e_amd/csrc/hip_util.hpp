// hip_util.hpp -- host-side HIP helpers shared by the engine's translation
// units (engine.hip, eval.hip): error checks that throw (turned into status
// codes at the C ABI) and an owning device buffer.
#pragma once

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

namespace kb2e {

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
// a configuration the engine does not run (KB2E_EUNSUPPORTED)
struct Unsupported : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define HIPCHK(expr)                                                                              \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess)                                                                     \
            throw ::kb2e::HipError(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" +     \
                                   std::string(__FILE__) + ":" + std::to_string(__LINE__));       \
    } while (0)

// hipMemset on the null stream, waited for: the engine's streams are
// non-blocking, so a kernel or copy queued on them next does not order after it.
inline void memset_sync(void* p, int v, size_t b) {
    HIPCHK(hipMemset(p, v, b));
    HIPCHK(hipStreamSynchronize(nullptr));
}

struct DevBuf {
    // the live-byte count an allocation is charged to: the context the engine is
    // working for (set by its entry points, kb2e_device_bytes); kept per buffer so
    // that a free later is returned to the same context
    static inline thread_local int64_t* tally_now = nullptr;
    void* p = nullptr;
    size_t bytes = 0;
    int64_t* tally = nullptr;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    void alloc(size_t b) {
        free();
        if (b == 0) b = 16;
        HIPCHK(hipMalloc(&p, b));
        tally = tally_now;
        if (tally) *tally += (int64_t)b;
        // zeroed: no kernel result may depend on what an earlier engine left in the
        // heap.  hipMemset runs on the null stream, which does not order against the
        // engine's non-blocking streams: wait for it here, or an upload queued next
        // on another stream (the filter table, the triples) can land before the
        // zeros and be wiped.
        memset_sync(p, 0, b);
        bytes = b;
    }
    void free() {
        if (p) {
            (void)hipFree(p);
            if (tally) *tally -= (int64_t)bytes;
        }
        p = nullptr;
        bytes = 0;
        tally = nullptr;
    }
    template <class T>
    T* as() const { return (T*)p; }
    ~DevBuf() { free(); }
};

}  // namespace kb2e
