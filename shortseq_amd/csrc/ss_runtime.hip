// ss_runtime.hip — C ABI runtime pieces: error strings, device selection, pinned staging buffers,
// and the host codec (per-object path) used by the drop-in Python objects.
#include <string.h>
#include <string>

#include "ss_internal.h"
#include "host_codec.h"

namespace {
thread_local std::string g_last_error;
}

int ss_fail(int code, const char* msg) {
    g_last_error = msg ? msg : "";
    return code;
}

int ss_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return SS_OK;
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return SS_EHIP;
}

extern "C" {

int ss_abi_version(void) { return SS_ABI_VERSION; }

const char* ss_last_error_string(void) { return g_last_error.c_str(); }

int ss_device_count(int* h_count) {
    if (!h_count) return ss_fail(SS_EARG, "null h_count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *h_count = 0;
        return ss_check(e, "hipGetDeviceCount");
    }
    *h_count = n;
    return SS_OK;
}

int ss_set_device(int device) { return ss_check(hipSetDevice(device), "hipSetDevice"); }

int ss_get_device(int* h_device) {
    if (!h_device) return ss_fail(SS_EARG, "null h_device");
    return ss_check(hipGetDevice(h_device), "hipGetDevice");
}

int ss_pinned_alloc(void** h_ptr, size_t bytes) {
    if (!h_ptr) return ss_fail(SS_EARG, "null h_ptr");
    return ss_check(hipHostMalloc(h_ptr, bytes, hipHostMallocDefault), "hipHostMalloc");
}

int ss_pinned_free(void* h_ptr) { return ss_check(hipHostFree(h_ptr), "hipHostFree"); }

int ss_host_encode(const uint8_t* h_seq, uint64_t L, uint64_t* h_words, ss_err* h_err) {
    return ssh::encode(h_seq, L, h_words, h_err);
}

void ss_host_decode(const uint64_t* h_words, uint64_t L, char* h_out) { ssh::decode(h_words, L, h_out); }

uint64_t ss_host_hamming(const uint64_t* h_a, const uint64_t* h_b, uint64_t L) {
    return ssh::hamming(h_a, h_b, L);
}

}  // extern "C"
