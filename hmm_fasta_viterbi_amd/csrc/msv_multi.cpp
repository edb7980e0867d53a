// msv_multi.cpp -- one batch over several GPUs from ONE process, with the score gather done by RCCL
// over xGMI (ncclCommInitAll, rccl.h:236; grouped ncclSend / ncclRecv, rccl.h:700-725).
//
// The reference has no multi-device path.  Sequences are independent, so the batch is cut
// into contiguous shards of ~equal residue count (msv_shard_bounds); one host thread per device
// uploads its shard (or, for page-locked residues, lets its kernel read them in place) and enqueues the
// longest-first order and ONE kernel launch on the device's stream;
// then a single RCCL group moves every shard's float scores into device 0's result buffer at the
// shard's offset (exact counts, no padding; rank 0's own shard goes through a self send/recv, so the
// exchange code runs even with one device), and one D2H returns them.  Only public msv.h entry points
// are used on the profiles; the context owns its streams, staging buffers and communicators.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <thread>
#include <vector>

#include "msv.h"

// msv_device.cpp (library-internal): whether page-locked residues are read in place for this model and size.
extern "C" bool msv_in_place_wins(const msv_profile* p, uint64_t bytes);
// msv_device.cpp (library-internal): msv_score_batch_device for page-locked host residues (zero-copy twin).
extern "C" msv_status msv_score_batch_host_residues(msv_profile* p, const uint8_t* d_residues, uint64_t residues_len,
                                         const uint64_t* d_offsets, uint64_t n, const uint32_t* d_order,
                                         float* d_scores, void* stream);

namespace {

constexpr uint64_t kChunkBytes = (1ull << 32) - (1ull << 20);  // per launch (msv_score_batch_device)

msv_status hip_status(hipError_t e) {
    if (e == hipSuccess) return MSV_OK;
    if (e == hipErrorOutOfMemory) return MSV_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return MSV_ERR_NO_DEVICE;
    return MSV_ERR_HIP;
}

#define MM_HIP(call)                                 \
    do {                                             \
        hipError_t e_ = (call);                      \
        if (e_ != hipSuccess) return hip_status(e_); \
    } while (0)
#define MM_NCCL(call)                                 \
    do {                                              \
        if ((call) != ncclSuccess) return MSV_ERR_RCCL; \
    } while (0)

template <typename T>
hipError_t grow(T*& p, size_t& cap, size_t need) {
    if (need <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t n = std::max<size_t>(need, 1);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), n * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
}

struct Rank {
    msv_profile* profile = nullptr;
    int device = -1;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    uint8_t* d_res = nullptr;
    size_t res_cap = 0;
    uint64_t* d_off = nullptr;
    size_t off_cap = 0;
    uint32_t* d_ord = nullptr;
    size_t ord_cap = 0;
    float* d_sc = nullptr;
    size_t sc_cap = 0;
    std::vector<uint64_t> h_off;  // rebased offsets of the shard's current launch
};

}  // namespace

struct msv_multi {
    std::vector<Rank> ranks;
    float* d_all = nullptr;  // device 0: every score, input order
    size_t all_cap = 0;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// msv_debug_multi_no_alias: make pinned_alias fail, so the copy fallback below runs (tests).
std::atomic<bool> g_no_alias{false};

// Device alias of page-locked host residues (nullptr for pageable memory): every rank's kernel then
// reads its shard in place over its own PCIe link instead of a staged copy (as msv_score_batch does).
// Called with the rank's device current.  ROCm documents hipHostMallocPortable as its default behaviour
// (page-locked memory is registered for every device), which covers msv_host_alloc and torch pin_memory;
// whether a non-owning device gets an alias has only run on one-GPU boxes here, so it is not relied on:
// when the call fails, nullptr sends the shard through the copy path (enqueue_shard), which
// msv_debug_multi_no_alias forces in the GPU tests (bitwise against one launch).
const uint8_t* pinned_alias(const uint8_t* host) {
    hipPointerAttribute_t at{};
    void* h = const_cast<uint8_t*>(host);
    if (!host || g_no_alias.load(std::memory_order_relaxed) || hipPointerGetAttributes(&at, h) != hipSuccess ||
        at.type != hipMemoryTypeHost) {
        (void)hipGetLastError();
        return nullptr;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<const uint8_t*>(d);
}

// Upload shard [first, last) to rank r's device and enqueue its order + kernel launches (one per
// < 4 GiB chunk) on the rank's stream.  Runs on the rank's own host thread.
msv_status enqueue_shard(Rank& r, const uint8_t* residues, const uint64_t* offsets, uint64_t first, uint64_t last) {
    DeviceGuard g(r.device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    const uint64_t cn = last - first;
    MM_HIP(grow(r.d_sc, r.sc_cap, cn));
    // (copied instead where the kernel would outrun the in-place reads: small models, large shards)
    const uint8_t* const zres =
        msv_in_place_wins(r.profile, offsets[last] - offsets[first]) ? pinned_alias(residues) : nullptr;
    uint64_t a = first;
    while (a < last) {  // chunks addressing < kChunkBytes residues each
        uint64_t b = a + 1;
        while (b < last && offsets[b + 1] - offsets[a] < kChunkBytes) ++b;
        if (offsets[b] - offsets[a] >= kChunkBytes) return MSV_ERR_SEQUENCE_TOO_LONG;
        const uint64_t n = b - a, base = offsets[a], bytes = offsets[b] - base;
        if (!zres) MM_HIP(grow(r.d_res, r.res_cap, std::max<uint64_t>(bytes, 1)));
        MM_HIP(grow(r.d_off, r.off_cap, n + 1));
        MM_HIP(grow(r.d_ord, r.ord_cap, n));
        r.h_off.resize(n + 1);
        for (uint64_t i = 0; i <= n; ++i) r.h_off[i] = offsets[a + i] - base;
        MM_HIP(hipMemcpyAsync(r.d_off, r.h_off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, r.stream));
        if (bytes && !zres) MM_HIP(hipMemcpyAsync(r.d_res, residues + base, bytes, hipMemcpyHostToDevice, r.stream));
        msv_status s = msv_order_longest_first(r.profile, r.d_off, n, r.d_ord, r.stream);
        if (s != MSV_OK) return s;
        const uint8_t* src = (zres && bytes) ? zres + base : (bytes ? r.d_res : nullptr);
        if (!src) {  // an all-empty chunk still needs one readable byte
            MM_HIP(grow(r.d_res, r.res_cap, 1));
            src = r.d_res;
        }
        s = (zres && bytes ? msv_score_batch_host_residues : msv_score_batch_device)(
            r.profile, src, std::max<uint64_t>(bytes, 1), r.d_off, n, r.d_ord, r.d_sc + (a - first), r.stream);
        if (s != MSV_OK) return s;
        // h_off (pageable) is rewritten by the next chunk: let this chunk's copy finish first
        if (b < last) MM_HIP(hipStreamSynchronize(r.stream));
        a = b;
    }
    return MSV_OK;
}

}  // namespace

extern "C" {

// Diagnostic (tests): on = every later msv_multi_score_batch copies page-locked shards instead of reading
// them in place, as if the device alias were unavailable.  Not in msv.h.
msv_status msv_debug_multi_no_alias(int on) {
    g_no_alias.store(on != 0, std::memory_order_relaxed);
    return MSV_OK;
}

void msv_multi_destroy(msv_multi* m) {
    if (!m) return;
    for (Rank& r : m->ranks) {
        if (r.device < 0) continue;
        DeviceGuard g(r.device);
        if (r.stream) (void)hipStreamSynchronize(r.stream);
        if (r.comm) (void)ncclCommDestroy(r.comm);
        (void)hipFree(r.d_res);
        (void)hipFree(r.d_off);
        (void)hipFree(r.d_ord);
        (void)hipFree(r.d_sc);
        if (r.stream) (void)hipStreamDestroy(r.stream);
    }
    if (!m->ranks.empty()) {
        DeviceGuard g(m->ranks[0].device);
        (void)hipFree(m->d_all);
    }
    delete m;
}

msv_status msv_multi_create(msv_profile* const* profiles, uint32_t n_profiles, msv_multi** out) {
    if (!profiles || n_profiles == 0 || !out) return MSV_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    std::vector<int> devs(n_profiles);
    for (uint32_t k = 0; k < n_profiles; ++k) {
        msv_kernel_info info;
        if (!profiles[k] || msv_profile_describe(profiles[k], &info) != MSV_OK) return MSV_ERR_INVALID_ARGUMENT;
        devs[k] = info.device;
        for (uint32_t j = 0; j < k; ++j)
            if (devs[j] == devs[k]) return MSV_ERR_INVALID_ARGUMENT;  // one RCCL rank per device
    }
    auto* m = new (std::nothrow) msv_multi;
    if (!m) return MSV_ERR_OUT_OF_MEMORY;
    m->ranks.resize(n_profiles);
    for (uint32_t k = 0; k < n_profiles; ++k) {
        Rank& r = m->ranks[k];
        r.profile = profiles[k];
        r.device = devs[k];
        DeviceGuard g(r.device);
        if (!g.ok || hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking) != hipSuccess) {
            msv_multi_destroy(m);
            return MSV_ERR_NO_DEVICE;
        }
    }
    // one communicator per device, ranks in the order given (rank 0 = profiles[0]'s device)
    std::vector<ncclComm_t> comms(n_profiles);
    if (ncclCommInitAll(comms.data(), static_cast<int>(n_profiles), devs.data()) != ncclSuccess) {
        msv_multi_destroy(m);
        return MSV_ERR_RCCL;
    }
    for (uint32_t k = 0; k < n_profiles; ++k) m->ranks[k].comm = comms[k];
    *out = m;
    return MSV_OK;
}

msv_status msv_multi_score_batch(msv_multi* m, const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                                 float* scores) {
    if (!m || (n && (!offsets || !scores))) return MSV_ERR_INVALID_ARGUMENT;
    if (n == 0) return MSV_OK;
    uint64_t maxL = 0;
    for (uint64_t s = 0; s < n; ++s) {
        if (offsets[s + 1] < offsets[s]) return MSV_ERR_INVALID_ARGUMENT;
        maxL = std::max<uint64_t>(maxL, offsets[s + 1] - offsets[s]);
    }
    if (offsets[n] > offsets[0] && !residues) return MSV_ERR_INVALID_ARGUMENT;
    const uint32_t R = static_cast<uint32_t>(m->ranks.size());
    std::vector<uint64_t> b(R + 1);
    msv_status s = msv_shard_bounds(offsets, n, R, b.data());
    if (s != MSV_OK) return s;
    for (Rank& r : m->ranks) {
        s = msv_profile_reserve_length(r.profile, maxL);
        if (s != MSV_OK) return s;
    }
    {
        DeviceGuard g(m->ranks[0].device);
        if (!g.ok) return MSV_ERR_NO_DEVICE;
        MM_HIP(grow(m->d_all, m->all_cap, n));
    }
    // 1. every rank uploads its shard and enqueues order + kernel, concurrently (one thread each)
    std::vector<msv_status> st(R, MSV_OK);
    std::vector<std::thread> workers;
    for (uint32_t k = 0; k < R; ++k) {
        if (b[k + 1] == b[k]) continue;
        workers.emplace_back([&, k] { st[k] = enqueue_shard(m->ranks[k], residues, offsets, b[k], b[k + 1]); });
    }
    for (auto& w : workers) w.join();
    for (uint32_t k = 0; k < R; ++k)
        if (st[k] != MSV_OK) return st[k];
    // 2. one RCCL group: shard k's scores -> device 0's buffer at offset b[k] (exact counts).  The
    //    calls switch the current device per rank; the guard gives the caller's back.  (Across two or
    //    more devices this exchange has not run on hardware yet: the test box has one GPU, where the
    //    group is rank 0's self send/recv.)
    DeviceGuard caller_device(m->ranks[0].device);
    if (!caller_device.ok) return MSV_ERR_NO_DEVICE;
    MM_NCCL(ncclGroupStart());
    for (uint32_t k = 0; k < R; ++k) {
        const uint64_t cnt = b[k + 1] - b[k];
        if (!cnt) continue;
        Rank& r = m->ranks[k];
        if (hipSetDevice(r.device) != hipSuccess ||
            ncclSend(r.d_sc, cnt, ncclFloat32, 0, r.comm, r.stream) != ncclSuccess ||
            hipSetDevice(m->ranks[0].device) != hipSuccess ||
            ncclRecv(m->d_all + b[k], cnt, ncclFloat32, static_cast<int>(k), m->ranks[0].comm,
                     m->ranks[0].stream) != ncclSuccess) {
            (void)ncclGroupEnd();
            return MSV_ERR_RCCL;
        }
    }
    MM_NCCL(ncclGroupEnd());
    // 3. one D2H from device 0, then each rank's latched kernel errors
    {
        DeviceGuard g(m->ranks[0].device);
        MM_HIP(hipMemcpyAsync(scores, m->d_all, n * sizeof(float), hipMemcpyDeviceToHost, m->ranks[0].stream));
        MM_HIP(hipStreamSynchronize(m->ranks[0].stream));
    }
    for (Rank& r : m->ranks) {
        s = msv_profile_check(r.profile, r.stream);
        if (s != MSV_OK) return s;
    }
    return MSV_OK;
}

}  // extern "C"
