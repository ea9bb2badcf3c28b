// ss_stage.hip — host-resident batches through the GPU (SURVEY §7 step 3, §8(b) "staging read
// batches in pinned memory").
//
// The Cython front and numpy callers hold reads in host memory.  ss_encode_host & co. stream such a
// batch through the device in fixed-size chunks with a ring of `nslots` pinned + device slots and
// three HIP streams, so that for chunks k+1, k, k-1 the H2D copy, the kernel and the D2H copy run
// at the same time (H2D and D2H use separate SDMA engines; PCIe is full duplex):
//
//   host thread : [stage in k+1 (pool memcpy)] [drain k-2 (pool memcpy)] ...
//   s_in        :   H2D k+1 ──ev_in──┐
//   s_k         :              kernel k ──ev_k──┐
//   s_out       :                          D2H k-1 ──ev_out──> host waits before the slot is reused
//
// Pageable user buffers go through the pinned slots with a multi-threaded memcpy (one core copies
// ~10 GB/s, below PCIe gen5 x16); user buffers that are already pinned (hipHostMalloc,
// torch.pin_memory) are DMA'd directly and the host copies disappear.  The slowest of PCIe, the
// staging copies and the kernel bounds the rate: this is the PCIe-inclusive path, never the
// device-resident roofline number.
#include <ctype.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "ss_internal.h"

namespace {

// Fixed pool of copy threads: copy() splits one memcpy into page-aligned parts, the calling
// thread takes part 0 and blocks until every part is done.
class CopyPool {
  public:
    // cpus: where the workers run (worker i on cpus[i % size]); empty = wherever the OS puts them
    CopyPool(int nthreads, const std::vector<int>& cpus) {
        for (int i = 0; i < nthreads; ++i) {
            th_.emplace_back([this, i] { worker(i); });
            if (!cpus.empty()) {
                cpu_set_t set;
                CPU_ZERO(&set);
                CPU_SET(cpus[i % cpus.size()], &set);
                (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof(set), &set);
            }
        }
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void copy(void* dst, const void* src, size_t n) {
        const int parts = (int)th_.size() + 1;
        if (n < (size_t(4) << 20) || parts == 1) {
            memcpy(dst, src, n);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            dst_ = (char*)dst;
            src_ = (const char*)src;
            n_ = n;
            parts_ = parts;
            pending_ = parts - 1;
            ++gen_;
        }
        cv_.notify_all();
        run_part(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
    }

  private:
    void run_part(int p) {
        const size_t per = ((n_ + parts_ - 1) / parts_ + 4095) & ~size_t(4095);
        const size_t a = std::min(n_, per * p), b = std::min(n_, a + per);
        if (b > a) memcpy(dst_ + a, src_ + a, b - a);
    }
    void worker(int i) {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            run_part(i + 1);
            std::lock_guard<std::mutex> g(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
    char* dst_ = nullptr;
    const char* src_ = nullptr;
    size_t n_ = 0;
    int parts_ = 1;
};

struct Slot {
    uint8_t* h_in = nullptr;    // pinned staging (pageable user input)
    uint8_t* h_out = nullptr;   // pinned staging (pageable user output)
    uint8_t* h_out2 = nullptr;
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* d_out2 = nullptr;
    uint64_t* d_fb = nullptr;   // the chunk's first-bad read (chunk-relative)
    uint64_t* h_fb = nullptr;   // pinned copy of it
    hipEvent_t ev_in = nullptr, ev_k = nullptr, ev_out = nullptr;
    hipEvent_t ev_h0 = nullptr, ev_k0 = nullptr, ev_o0 = nullptr;   // stage starts (ss_stager_set_timing)
    bool busy = false, timed = false;
    uint64_t base = 0, m = 0;
};

// One host batch operation: per-read byte counts of the input and the (up to two) outputs, and the
// kernel launch for a chunk of m reads already in device memory.
struct HostOp {
    const uint8_t* h_in;
    size_t in_bpr;
    uint8_t* h_out;
    size_t out_bpr;
    uint8_t* h_out2;      // optional second output (distances)
    size_t out2_bpr;
    bool has_fb;
    int (*launch)(const HostOp& op, const uint8_t* d_in, uint64_t m, uint8_t* d_out, uint8_t* d_out2,
                  uint64_t* d_fb, hipStream_t s);
    // launch parameters
    uint32_t L, wpr;
    uint64_t stride;
    const uint64_t* d_ref;
};

bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

}  // namespace

struct ss_stager {
    int device = 0;
    uint64_t chunk_bytes = 0;
    std::vector<Slot> slots;
    hipStream_t s_in = nullptr, s_k = nullptr, s_out = nullptr;
    CopyPool* pool = nullptr;
    bool out2_ready = false;
    // placement: copy threads, CPUs in the process's affinity mask, the GPU's NUMA
    // node (-1: unknown), CPUs the copy threads were pinned to (the node's CPUs in the mask; 0: none)
    int copy_threads = 0, affinity_cpus = 0, numa_node = -1, pinned_cpus = 0;
    // stage split (ss_stager_set_timing): host ms of the pageable -> pinned copies, the pinned ->
    // pageable copies and the waits on the D2H events; device ms of H2D, kernel, D2H (event pairs per
    // chunk); calls since the last ss_stager_stats
    bool timing = false;
    double ms[6] = {};
    uint64_t calls = 0;
};

namespace {

void free_stager(ss_stager* st) {
    if (!st) return;
    (void)hipSetDevice(st->device);
    if (st->s_in) (void)hipStreamSynchronize(st->s_in);
    if (st->s_k) (void)hipStreamSynchronize(st->s_k);
    if (st->s_out) (void)hipStreamSynchronize(st->s_out);
    for (Slot& s : st->slots) {
        if (s.h_in) (void)hipHostFree(s.h_in);
        if (s.h_out) (void)hipHostFree(s.h_out);
        if (s.h_out2) (void)hipHostFree(s.h_out2);
        if (s.h_fb) (void)hipHostFree(s.h_fb);
        if (s.d_in) (void)hipFree(s.d_in);
        if (s.d_out) (void)hipFree(s.d_out);
        if (s.d_out2) (void)hipFree(s.d_out2);
        if (s.d_fb) (void)hipFree(s.d_fb);
        if (s.ev_in) (void)hipEventDestroy(s.ev_in);
        if (s.ev_k) (void)hipEventDestroy(s.ev_k);
        if (s.ev_out) (void)hipEventDestroy(s.ev_out);
        if (s.ev_h0) (void)hipEventDestroy(s.ev_h0);
        if (s.ev_k0) (void)hipEventDestroy(s.ev_k0);
        if (s.ev_o0) (void)hipEventDestroy(s.ev_o0);
    }
    if (st->s_in) (void)hipStreamDestroy(st->s_in);
    if (st->s_k) (void)hipStreamDestroy(st->s_k);
    if (st->s_out) (void)hipStreamDestroy(st->s_out);
    delete st->pool;
    delete st;
}

int ensure_out2(ss_stager* st) {
    if (st->out2_ready) return SS_OK;
    for (Slot& s : st->slots) {
        int rc = ss_check(hipHostMalloc((void**)&s.h_out2, st->chunk_bytes, hipHostMallocDefault), "hipHostMalloc");
        if (!rc) rc = ss_check(hipMalloc((void**)&s.d_out2, st->chunk_bytes), "hipMalloc");
        if (rc) return rc;
    }
    st->out2_ready = true;
    return SS_OK;
}

// Wait for a slot's chunk, move its outputs to the user buffers, fold in its first-bad read.
using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

int drain(ss_stager* st, Slot& s, const HostOp& op, bool out_pinned, bool out2_pinned, uint64_t* first_bad) {
    if (!s.busy) return SS_OK;
    s.busy = false;
    auto t0 = Clock::now();
    int rc = ss_check(hipEventSynchronize(s.ev_out), "hipEventSynchronize(d2h)");
    if (rc) return rc;
    st->ms[5] += ms_since(t0);
    if (s.timed) {     // every event of the chunk has completed (the D2H waited on the kernel, it on the H2D)
        float a = 0, b = 0, c = 0;
        if (hipEventElapsedTime(&a, s.ev_h0, s.ev_in) == hipSuccess && hipEventElapsedTime(&b, s.ev_k0, s.ev_k) == hipSuccess &&
            hipEventElapsedTime(&c, s.ev_o0, s.ev_out) == hipSuccess) {
            st->ms[2] += a;
            st->ms[3] += b;
            st->ms[4] += c;
        } else {
            (void)hipGetLastError();
        }
        s.timed = false;
    }
    t0 = Clock::now();
    if (!out_pinned) st->pool->copy(op.h_out + s.base * op.out_bpr, s.h_out, s.m * op.out_bpr);
    if (op.h_out2 && !out2_pinned) st->pool->copy(op.h_out2 + s.base * op.out2_bpr, s.h_out2, s.m * op.out2_bpr);
    st->ms[1] += ms_since(t0);
    if (op.has_fb && *s.h_fb != ~0ull && *first_bad == ~0ull) *first_bad = s.base + *s.h_fb;
    return SS_OK;
}

int run(ss_stager* st, const HostOp& op, uint64_t n, uint64_t* h_first_bad) {
    if (!st) return ss_fail(SS_EARG, "null stager");
    if (h_first_bad) *h_first_bad = ~0ull;
    if (n == 0) return SS_OK;
    int rc = ss_check(hipSetDevice(st->device), "hipSetDevice");
    if (rc) return rc;
    if (op.h_out2 && (rc = ensure_out2(st))) return rc;
    const size_t per = std::max({op.in_bpr, op.out_bpr, op.h_out2 ? op.out2_bpr : size_t(1)});
    const uint64_t rpc = std::max<uint64_t>(1, st->chunk_bytes / per);
    if (per > st->chunk_bytes) return ss_fail(SS_EARG, "stager chunk smaller than one read");
    const bool in_pinned = is_pinned(op.h_in);
    const bool out_pinned = is_pinned(op.h_out);
    const bool out2_pinned = op.h_out2 && is_pinned(op.h_out2);
    uint64_t first_bad = ~0ull;
    const uint32_t ns = (uint32_t)st->slots.size();
    const uint64_t nchunks = (n + rpc - 1) / rpc;
    if (st->timing) ++st->calls;
    for (uint64_t k = 0; k < nchunks && !rc; ++k) {
        Slot& s = st->slots[k % ns];
        if ((rc = drain(st, s, op, out_pinned, out2_pinned, &first_bad))) break;
        s.base = k * rpc;
        s.m = std::min(rpc, n - s.base);
        const uint8_t* src = op.h_in + s.base * op.in_bpr;
        const size_t in_b = s.m * op.in_bpr;
        if (!in_pinned) {
            const auto t0 = Clock::now();
            st->pool->copy(s.h_in, src, in_b);
            st->ms[0] += ms_since(t0);
            src = s.h_in;
        }
        s.timed = st->timing && s.ev_h0;
        if (s.timed) rc = ss_check(hipEventRecord(s.ev_h0, st->s_in), "hipEventRecord");
        if (!rc) rc = ss_check(hipMemcpyAsync(s.d_in, src, in_b, hipMemcpyHostToDevice, st->s_in), "H2D");
        if (!rc) rc = ss_check(hipEventRecord(s.ev_in, st->s_in), "hipEventRecord");
        if (!rc) rc = ss_check(hipStreamWaitEvent(st->s_k, s.ev_in, 0), "hipStreamWaitEvent");
        if (!rc && s.timed) rc = ss_check(hipEventRecord(s.ev_k0, st->s_k), "hipEventRecord");
        if (!rc) rc = op.launch(op, s.d_in, s.m, s.d_out, s.d_out2, s.d_fb, st->s_k);
        if (!rc) rc = ss_check(hipEventRecord(s.ev_k, st->s_k), "hipEventRecord");
        if (!rc) rc = ss_check(hipStreamWaitEvent(st->s_out, s.ev_k, 0), "hipStreamWaitEvent");
        if (!rc && s.timed) rc = ss_check(hipEventRecord(s.ev_o0, st->s_out), "hipEventRecord");
        if (!rc) {
            uint8_t* dst = out_pinned ? op.h_out + s.base * op.out_bpr : s.h_out;
            rc = ss_check(hipMemcpyAsync(dst, s.d_out, s.m * op.out_bpr, hipMemcpyDeviceToHost, st->s_out), "D2H");
        }
        if (!rc && op.h_out2) {
            uint8_t* dst = out2_pinned ? op.h_out2 + s.base * op.out2_bpr : s.h_out2;
            rc = ss_check(hipMemcpyAsync(dst, s.d_out2, s.m * op.out2_bpr, hipMemcpyDeviceToHost, st->s_out), "D2H");
        }
        if (!rc && op.has_fb)
            rc = ss_check(hipMemcpyAsync(s.h_fb, s.d_fb, sizeof(uint64_t), hipMemcpyDeviceToHost, st->s_out), "D2H");
        if (!rc) rc = ss_check(hipEventRecord(s.ev_out, st->s_out), "hipEventRecord");
        s.busy = true;
    }
    // drain in chunk order (first_bad is the first flagged chunk in input order)
    const uint64_t k0 = nchunks > ns ? nchunks - ns : 0;
    for (uint64_t k = k0; k < nchunks; ++k) {
        int r2 = drain(st, st->slots[k % ns], op, out_pinned, out2_pinned, &first_bad);
        if (!rc) rc = r2;
    }
    if (h_first_bad) *h_first_bad = first_bad;
    return rc;
}

int launch_encode(const HostOp& op, const uint8_t* d_in, uint64_t m, uint8_t* d_out, uint8_t* d_out2,
                  uint64_t* d_fb, hipStream_t s) {
    return ss_encode_fixed_impl(d_in, m, op.L, op.stride, (uint64_t*)d_out, op.wpr, d_fb, op.d_ref,
                                (uint32_t*)d_out2, s);
}

int launch_decode(const HostOp& op, const uint8_t* d_in, uint64_t m, uint8_t* d_out, uint8_t*, uint64_t*,
                  hipStream_t s) {
    return ss_decode_fixed((const uint64_t*)d_in, m, op.L, op.wpr, d_out, op.stride, s);
}

// The copy threads' CPUs: the GPU's NUMA node's CPUs that the process's affinity mask allows
// (ss_gpu_numa_cpus); empty when the node is unknown, the intersection is empty, or
// SHORTSEQ_STAGE_PIN=0.  Fills the stager's placement fields.
std::vector<int> placement(ss_stager* st) {
    int node = -1, allowed = 0;
    std::vector<int> mine = ss_gpu_numa_cpus(st->device, &node, &allowed);
    st->affinity_cpus = allowed;
    st->numa_node = node;
    const char* env = getenv("SHORTSEQ_STAGE_PIN");
    if (node < 0 || (env && env[0] == '0')) return {};
    st->pinned_cpus = (int)mine.size();
    return mine;
}

}  // namespace

// CPUs of a sysfs cpulist ("0-7,64-71")
static std::vector<int> parse_cpulist(const char* path) {
    std::vector<int> out;
    FILE* f = fopen(path, "r");
    if (!f) return out;
    char buf[4096];
    const size_t len = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[len] = 0;
    for (char* p = buf; *p;) {
        char* e = nullptr;
        const long a = strtol(p, &e, 10);
        if (e == p) break;
        long b = a;
        p = e;
        if (*p == '-') {
            b = strtol(p + 1, &e, 10);
            p = e;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) out.push_back((int)c);
        while (*p == ',' || *p == '\n' || *p == ' ') ++p;
    }
    return out;
}

std::vector<int> ss_gpu_numa_cpus(int device, int* node_out, int* allowed_out) {
    cpu_set_t mask;
    CPU_ZERO(&mask);
    std::vector<int> allowed;
    if (sched_getaffinity(0, sizeof(mask), &mask) == 0)
        for (int c = 0; c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &mask)) allowed.push_back(c);
    if (allowed_out) *allowed_out = (int)allowed.size();
    if (node_out) *node_out = -1;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) {
        (void)hipGetLastError();
        return {};
    }
    for (char* q = bus; *q; ++q) *q = (char)tolower(*q);
    char path[256];
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE* f = fopen(path, "r");
    int node = -1;
    if (f) {
        if (fscanf(f, "%d", &node) != 1) node = -1;
        fclose(f);
    }
    if (node_out) *node_out = node;
    if (node < 0) return {};
    snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
    std::vector<int> mine;
    for (int c : parse_cpulist(path))
        if (std::find(allowed.begin(), allowed.end(), c) != allowed.end()) mine.push_back(c);
    return mine;
}

extern "C" {

int ss_stager_set_timing(ss_stager* st, int on) {
    if (!st) return ss_fail(SS_EARG, "null stager");
    int rc = ss_check(hipSetDevice(st->device), "hipSetDevice");
    for (Slot& s : st->slots) {
        if (rc || !on || s.ev_h0) break;
        rc = ss_check(hipEventCreate(&s.ev_h0), "hipEventCreate");
        if (!rc) rc = ss_check(hipEventCreate(&s.ev_k0), "hipEventCreate");
        if (!rc) rc = ss_check(hipEventCreate(&s.ev_o0), "hipEventCreate");
    }
    if (rc) return rc;
    st->timing = on != 0;
    return SS_OK;
}

int ss_stager_stats(ss_stager* st, double* h_ms, int32_t* h_info) {
    if (!st || !h_ms || !h_info) return ss_fail(SS_EARG, "null argument");
    const double k = st->calls ? 1.0 / (double)st->calls : 0.0;
    for (int i = 0; i < 6; ++i) {
        h_ms[i] = st->ms[i] * k;
        st->ms[i] = 0;
    }
    h_info[0] = st->copy_threads;
    h_info[1] = st->affinity_cpus;
    h_info[2] = st->numa_node;
    h_info[3] = st->pinned_cpus;
    st->calls = 0;
    return SS_OK;
}

int ss_stager_create(int device, uint64_t chunk_bytes, uint32_t nslots, uint32_t copy_threads,
                     ss_stager** h_out) {
    if (!h_out) return ss_fail(SS_EARG, "null h_out");
    *h_out = nullptr;
    if (nslots < 2 || nslots > 16) return ss_fail(SS_EARG, "nslots must be in 2..16");
    if (chunk_bytes < 4096 || chunk_bytes > (uint64_t(1) << 34)) return ss_fail(SS_EARG, "chunk_bytes out of range");
    if (copy_threads > 64) return ss_fail(SS_EARG, "copy_threads must be <= 64");
    chunk_bytes = (chunk_bytes + 4095) & ~uint64_t(4095);
    ss_stager* st = new (std::nothrow) ss_stager();
    if (!st) return ss_fail(SS_ENOMEM, "ss_stager");
    st->device = device;
    st->chunk_bytes = chunk_bytes;
    int rc = ss_check(hipSetDevice(device), "hipSetDevice");
    if (!rc) rc = ss_check(hipStreamCreateWithFlags(&st->s_in, hipStreamNonBlocking), "hipStreamCreate");
    if (!rc) rc = ss_check(hipStreamCreateWithFlags(&st->s_k, hipStreamNonBlocking), "hipStreamCreate");
    if (!rc) rc = ss_check(hipStreamCreateWithFlags(&st->s_out, hipStreamNonBlocking), "hipStreamCreate");
    st->slots.resize(nslots);
    for (uint32_t i = 0; i < nslots && !rc; ++i) {
        Slot& s = st->slots[i];
        rc = ss_check(hipHostMalloc((void**)&s.h_in, chunk_bytes, hipHostMallocDefault), "hipHostMalloc");
        if (!rc) rc = ss_check(hipHostMalloc((void**)&s.h_out, chunk_bytes, hipHostMallocDefault), "hipHostMalloc");
        if (!rc) rc = ss_check(hipHostMalloc((void**)&s.h_fb, sizeof(uint64_t), hipHostMallocDefault), "hipHostMalloc");
        if (!rc) rc = ss_check(hipMalloc((void**)&s.d_in, chunk_bytes), "hipMalloc");
        if (!rc) rc = ss_check(hipMalloc((void**)&s.d_out, chunk_bytes), "hipMalloc");
        if (!rc) rc = ss_check(hipMalloc((void**)&s.d_fb, sizeof(uint64_t)), "hipMalloc");
        // (timing-capable: they also end the stage spans of ss_stager_set_timing)
        if (!rc) rc = ss_check(hipEventCreate(&s.ev_in), "hipEventCreate");
        if (!rc) rc = ss_check(hipEventCreate(&s.ev_k), "hipEventCreate");
        if (!rc) rc = ss_check(hipEventCreate(&s.ev_out), "hipEventCreate");
    }
    if (rc) {
        free_stager(st);
        return rc;
    }
    st->copy_threads = (int)copy_threads;
    const std::vector<int> cpus = placement(st);
    st->pool = new (std::nothrow) CopyPool((int)copy_threads, cpus);
    if (!st->pool) {
        free_stager(st);
        return ss_fail(SS_ENOMEM, "copy pool");
    }
    *h_out = st;
    return SS_OK;
}

int ss_stager_destroy(ss_stager* st) {
    free_stager(st);
    return SS_OK;
}

int ss_encode_host(ss_stager* st, const uint8_t* h_ascii, uint64_t n, uint32_t L, uint64_t stride,
                   uint64_t* h_words, uint32_t wpr, uint64_t* h_first_bad) {
    if (n && (!h_ascii || !h_words)) return ss_fail(SS_EARG, "null buffer");
    if (!h_first_bad) return ss_fail(SS_EARG, "h_first_bad is required");
    if (L == 0 || L > SS_MAX_NT || stride < L || wpr == 0 || wpr > 32) return ss_fail(SS_EARG, "bad L / stride / wpr");
    HostOp op{h_ascii, (size_t)stride, (uint8_t*)h_words, (size_t)8 * wpr, nullptr, 0, true, launch_encode,
              L, wpr, stride, nullptr};
    return run(st, op, n, h_first_bad);
}

int ss_encode_hamming_ref_host(ss_stager* st, const uint8_t* h_ascii, uint64_t n, uint32_t L, uint64_t stride,
                               uint64_t* h_words, uint32_t wpr, const uint64_t* d_ref_words, uint32_t* h_out,
                               uint64_t* h_first_bad) {
    if (n && (!h_ascii || !h_words || !h_out || !d_ref_words)) return ss_fail(SS_EARG, "null buffer");
    if (!h_first_bad) return ss_fail(SS_EARG, "h_first_bad is required");
    if (L == 0 || L > SS_MAX_NT || stride < L || wpr == 0 || wpr > 32) return ss_fail(SS_EARG, "bad L / stride / wpr");
    HostOp op{h_ascii, (size_t)stride, (uint8_t*)h_words, (size_t)8 * wpr, (uint8_t*)h_out, sizeof(uint32_t),
              true, launch_encode, L, wpr, stride, d_ref_words};
    return run(st, op, n, h_first_bad);
}

int ss_decode_host(ss_stager* st, const uint64_t* h_words, uint64_t n, uint32_t L, uint32_t wpr,
                   uint8_t* h_ascii, uint64_t stride) {
    if (n && (!h_ascii || !h_words)) return ss_fail(SS_EARG, "null buffer");
    if (L == 0 || L > SS_MAX_NT || stride < L || wpr == 0 || wpr > 32) return ss_fail(SS_EARG, "bad L / stride / wpr");
    HostOp op{(const uint8_t*)h_words, (size_t)8 * wpr, h_ascii, (size_t)stride, nullptr, 0, false, launch_decode,
              L, wpr, stride, nullptr};
    return run(st, op, n, nullptr);
}

}  // extern "C"
