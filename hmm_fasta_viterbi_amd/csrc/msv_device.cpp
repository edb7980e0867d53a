// msv_device.cpp -- C-ABI of the device hot path (msv.h) on the HIP runtime.
//
// Replaces the per-call OpenCL orchestration of MSV_HMM::parallel_run_on_sequence
// (algorithms/MSV_HMM.cpp:269-430: a context, 23 buffers, a JIT program build and 9-14 kernel
// launches per residue, for every sequence) with: one device-resident profile built once
// (kernel-layout emission table + per-length transition table), and one persistent kernel
// launch per batch.  Status codes are returned, never printed-and-continued (:198-203).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "launch_ring.h"
#include "msv.h"
#include "msv_kernel.h"

namespace {

constexpr uint32_t kDefaultMaxLength = 131072;
constexpr uint32_t kOrderBins = 4096;  // lengths >= 4095 share the longest bin
// Every launch of one profile takes the next of kLaunchSlots device counter pairs {next index, waves
// left} (and, for the longest-first order, the next histogram), so launches on different streams
// never share a counter; a slot is reused only after its previous launch (an event wait when the
// streams differ).  d_words: [2k, 2k+1] = slot k's counters, [kErrWord] = sticky error bits,
// [kErrWord + 1 + a] = the error bits of asynchronous staging slot a (msv_score_batch_async),
// [kHostErrWord] = the error bits of synchronous host calls (msv_score_batch), which report and clear only
// their own: bits latched by msv_score_batch_device launches stay for msv_profile_check.
constexpr int kLaunchSlots = 8;
constexpr int kAsyncSlots = 3;
constexpr int kErrWord = 2 * kLaunchSlots;
constexpr int kHostErrWord = kErrWord + 1 + kAsyncSlots;
constexpr int kWords = kHostErrWord + 1;
// Every launch addresses < 2^32 residue bytes.
constexpr uint64_t kChunkBytes = (1ull << 32) - (1ull << 20);
// Host batches of at least this many residues are scored as a copy/compute pipeline of pieces.
constexpr uint64_t kPipelineMin = 4ull << 20;
// Small host calls (pageable residues of at most kSmallCall bytes, at most kSmallCall sequences -- the
// reference's one-sequence-per-call pattern): residues staged behind the offsets in the pinned offsets
// buffer and sent in ONE H2D; pageable scores written by the kernel into pinned staging (no D2H).
constexpr uint64_t kSmallCall = 1ull << 20;
// Page-locked residues are read in place unless the model has fewer than kInPlaceMinStates states and the
// batch at least kInPlaceAnyBytes residues (msv_score_batch).
constexpr uint32_t kInPlaceMinStates = 300;
constexpr uint64_t kInPlaceAnyBytes = 16ull << 20;

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

// MSV_HMM::init_transitions_depend_on_seq (MSV_HMM.cpp:59-64) for every length < n, with the
// host's logf (never a device logf, so the per-sequence constants are the reference's bits).
// Returns a copy of the first n entries: the shared cache may grow under another thread (one host
// thread per device in msv_score_batch_multi), so nothing refers into it outside the lock.
std::vector<float2> host_length_table(uint32_t n) {
    static std::mutex mu;
    static std::vector<float2> table;
    std::lock_guard<std::mutex> lock(mu);
    if (table.size() < n) {
        const size_t old = table.size();
        table.resize(n);
        for (size_t L = old; L < n; ++L) {
            float loop, move;
            msv_sequence_transitions(L, &loop, &move);
            table[L] = make_float2(loop, move);
        }
    }
    return std::vector<float2>(table.begin(), table.begin() + n);
}

template <typename T>
hipError_t ensure(T*& p, size_t& cap, size_t need) {
    if (need <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t n = std::max<size_t>(need, 1);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), n * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
}

msv_status hip_status(hipError_t e) {
    if (e == hipSuccess) return MSV_OK;
    if (e == hipErrorOutOfMemory) return MSV_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return MSV_ERR_NO_DEVICE;
    return MSV_ERR_HIP;
}

#define MSV_HIP(call)                                    \
    do {                                                 \
        hipError_t e_ = (call);                          \
        if (e_ != hipSuccess) return hip_status(e_);     \
    } while (0)

// Estimated issue cost of one row for one sequence: 2.5 VALU per state-slot plus the per-row
// specials/reduction, times the lanes a sequence occupies.  A BIG table costs little with one
// sequence per wave (G = 64: wave-uniform LDS/L2 row split) and a lot with 2-4 sequences per wave
// (generic loads with per-lane address selects); measured on 2405.hmm: 7.4 vs 10.5 ms.
// A split table (the lane's last S - SA states read from L2 every row) costs the B-table address and
// loads per row and no class branch, so it also runs two sequences per wave (G = 32).
double variant_cost(const msvk::Variant& v) {
    // (G = 64 BIG: 1.15 -- 1901.hmm's 64 x 32 row-class plan measured 1.12 / 2.20 ms against 0.97 / 1.99 ms
    // for the 64 x 34 split plan at 3 / 2048 sequences, profiles/r02_latency_plans.jsonl)
    const double big = !v.big ? 1.0 : (v.G == 64 ? 1.15 : 1.6);
    // G = 64: + permlane32 step, scalar bookkeeping
    const double row = (v.G == 64 ? 36.0 : 26.0) + (v.sa ? 2.0 : 0.0);
    return (2.5 * v.S + row) * v.G * big * (v.pf == 2 ? 1.0 : 1.05) * (v.streams == 2 ? 1.15 : 1.0);
}

// Latency plan for small batches: one sequence per wave (G = 64) so a row is ~40% of the
// instructions of a 16-lane row; the cheapest such variant covering the model (non-BIG if any).
const msvk::Variant* pick_latency_variant(uint32_t states) {
    int count = 0;
    const msvk::Variant* all = msvk::variants(&count);
    const msvk::Variant* best = nullptr;
    for (int i = 0; i < count; ++i) {
        const msvk::Variant& v = all[i];
        if (v.G != 64 || static_cast<uint32_t>(v.G * v.S) < states) continue;
        if (!best || variant_cost(v) < variant_cost(*best)) best = &v;
    }
    return best;
}

// Mid plan for batches between the latency plan's and one round of the main grid: two sequences per
// wave (G = 32), the cheapest plain (LDS-table, one-stream) variant covering the model.
const msvk::Variant* pick_mid_variant(uint32_t states) {
    int count = 0;
    const msvk::Variant* all = msvk::variants(&count);
    const msvk::Variant* best = nullptr;
    for (int i = 0; i < count; ++i) {
        const msvk::Variant& v = all[i];
        if (v.G != 32 || v.streams != 1 || v.big || v.sa || static_cast<uint32_t>(v.G * v.S) < states) continue;
        if (!best || variant_cost(v) < variant_cost(*best)) best = &v;
    }
    return best;
}

// `narrow`: 4-lane groups may be picked.  Their rows are long (16 sequences per wave), which the issue
// model rewards and which wins once the SIMDs are full, so they are the throughput plan of the smallest
// profiles (100.hmm x 100k: g4_s28 0.339 vs g16_s8 0.521 ms, x 1M 3.08 vs 4.11 ms) while batches that
// leave the SIMDs part-empty keep a 16-lane plan (x 10k: 0.138 vs 0.099 ms; install_variant).  8-lane
// groups stay tuning candidates: on 200.hmm g8_s32 against g16_s16 was 6% slower at 100k, 2% faster
// at 1M (profiles/r02_small_profiles.jsonl).
// A whole-row emission ring (PF = S/4: the next row's chunks requested during this row's epilogue) on
// 16 waves, for 16-lane rows of 16-32 states.
static bool whole_row_ring(const msvk::Variant& v) {
    return v.G == 16 && v.streams == 1 && !v.big && !v.sa && v.pf * 4 == v.S && v.S >= 16 && v.S <= 32;
}

// `whole_row`: whole-row-ring variants are preferred where they exist -- on full batches 1-5% faster
// than the PF-2 ones (200/300/400/500.hmm x 100k: 0.692/0.827/1.051/1.196 vs 0.708/0.837/1.094/1.259 ms),
// while below a round of the grid the PF-2 ones hold (500.hmm x 10k: 0.229 vs 0.197 ms;
// profiles/r02_whole_row_rings.jsonl), so those stay the plan of smaller batches (install_variant).
const msvk::Variant* pick_variant(uint32_t states, bool narrow, bool whole_row = false) {
    int count = 0;
    const msvk::Variant* all = msvk::variants(&count);
    const msvk::Variant* best = nullptr;
    auto cost = [&](const msvk::Variant& v) { return variant_cost(v) * (whole_row && whole_row_ring(v) ? 0.9 : 1.0); };
    for (int i = 0; i < count; ++i) {
        const msvk::Variant& v = all[i];
        if (static_cast<uint32_t>(v.G * v.S) < states) continue;
        // (not for tables of fewer than 80 states: a 28-state lane row would be mostly padding, unmeasured)
        if (v.G < 16 && !(narrow && v.G == 4 && states >= 80)) continue;
        if (!best || cost(v) < cost(*best)) best = &v;
    }
    return best;
}

// Launch slots of one profile (see kLaunchSlots and launch_ring.h).
using LaunchRing = msvrt::LaunchRing<kLaunchSlots>;

}  // namespace

// One kernel instantiation with its emission table (in that variant's layout) and grid.
struct Plan {
    const msvk::Variant* v = nullptr;
    const msvk::CoopVariant* cv = nullptr;  // the cooperative plan (msv_coop.hip) instead of a variant
    float4* d_etab = nullptr;
    int blocks = 0;  // persistent grid size
    int groups_per_block = 0;
};

struct msv_profile {
    int device = 0;
    uint32_t model_length = 0;  // LENG + 1
    Plan main;                    // throughput plan (every launch unless the batch is small)
    Plan lat;                     // latency plan for small batches (G = 64), may equal main's variant
    Plan mid;                     // mid-size batches (G = 32), large G = 16 profiles only
    Plan fused;                   // the table in another profile's latency layout (fused grid launches)
    Plan coop;                    // one sequence per workgroup, the row over its waves (msv_coop.hip)
    Plan coop_fused;              // the table in another profile's cooperative layout (fused grid launches)
    uint64_t coop_max_n = 0;      // batches up to this many sequences take the cooperative plan
    bool force = false;           // msv_profile_set_variant: main plan for every batch size
    uint64_t lat_max_n = 0;       // batches up to this many sequences take the latency plan
    uint64_t mid_max_n = 0;       // batches above lat_max_n and up to this many take the mid plan
    float tr_B_Mk = 0, tr_E_C = 0, tr_E_J = 0;
    std::vector<float> emission_scores;  // host copy [20][model_length] (for re-layout)
    float2* d_lentab = nullptr;
    uint32_t lentab_n = 0;
    uint32_t* d_words = nullptr;  // kLaunchSlots x {dequeue counter, waves still running}, sticky error bits
    uint32_t* d_hist = nullptr;   // kLaunchSlots longest-first counting-sort scratches [hist | cursors]
    std::array<bool, kLaunchSlots> hist_dirty{};  // histogram not known to be zero (fresh, failed launch)
    uint8_t* d_dummy = nullptr;   // a readable residue byte for batches with no residues
    LaunchRing kernels, orders;   // launch slots of the MSV kernel and of the order sort
    hipStream_t stream = nullptr;
    hipStream_t bound = nullptr;  // msv_profile_bind_stream: a caller stream guaranteed alive while bound
    // host-API pipeline (msv_score_batch): a second compute stream, a copy stream, piece events,
    // and pinned staging for the rebased offsets
    hipStream_t stream2 = nullptr, copy_stream = nullptr;
    hipStream_t offsets_stream = nullptr;  // msv_score_batch_async: the offsets' H2D, beside the residues'
    std::vector<hipEvent_t> events;
    uint64_t* h_off = nullptr;
    size_t h_off_cap = 0;
    float* h_sc = nullptr;  // pinned score staging of small calls with pageable destinations
    size_t h_sc_cap = 0;
    uint32_t pipe_first_den = 4, pipe_growth = 2;  // piece sizes: total / first_den, then x growth
    uint32_t pipe_streams = 2;                      // compute streams the pieces alternate over
    bool zero_copy = true;  // page-locked residues read in place (msv_debug_set_zero_copy turns it off)
    bool zc_wide = true;    // ... by the wide-block twins of residue-block variants (msv_debug_set_zero_copy 2: off)
    // msv_score_batch_async: kAsyncSlots staging sets, so the H2D of one call runs under the kernel
    // of the call before it
    struct AsyncSlot {
        uint8_t* d_res = nullptr;
        size_t res_cap = 0;
        uint64_t* d_off = nullptr;
        size_t off_cap = 0;
        float* d_sc = nullptr;
        size_t sc_cap = 0;
        uint32_t* d_ord = nullptr;
        size_t ord_cap = 0;
        uint64_t* h_off = nullptr;  // pinned rebased offsets
        size_t h_cap = 0;
        uint32_t* h_err = nullptr;  // pinned copy of the slot's error word
        const float* direct = nullptr;  // page-locked destination written by the kernel (errors: scan)
        uint64_t n = 0;
        hipEvent_t copied = nullptr, done = nullptr, off_copied = nullptr;
        uint64_t ticket = 0;
        bool pending = false;
    } async[kAsyncSlots];
    uint64_t next_ticket = 1;
    // host-API staging
    uint8_t* d_res = nullptr;
    size_t d_res_cap = 0;
    uint64_t* d_off = nullptr;
    size_t d_off_cap = 0;
    float* d_scores = nullptr;
    size_t d_scores_cap = 0;
    uint32_t* d_order = nullptr;  // msv_score_fasta_device's longest-first order
    size_t d_order_cap = 0;
    uint64_t* d_stamps = nullptr;  // diagnostic timeline buffer (tools only), or nullptr
    bool stamp_clock = false;      // d_stamps is for the CLOCK twins (kStampWords per wave: bench.py clock_GHz)
    hipEvent_t time_start = nullptr, time_stop = nullptr;  // msv_debug_time_next_launch (one launch)
    hipEvent_t done = nullptr;     // grid API: joins this profile's stream back to the caller's
    hipStream_t shared = nullptr;  // shared_stream(device) once a host grid call used it
};


// One stream per device that the library never destroys: host grid calls launch on it, so every
// profile of the grid may leave its slot event unrecorded (a per-profile event record is a packet on
// the stream: 24 of them put ~115 us between a fused grid launch and its scores' D2H).
static hipStream_t shared_stream(int device) {
    static std::mutex mu;
    static std::map<int, hipStream_t> streams;
    std::lock_guard<std::mutex> lock(mu);
    auto it = streams.find(device);
    if (it != streams.end()) return it->second;
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
    streams[device] = st;
    return st;
}

// Streams on which a launch may leave its slot event unrecorded (LaunchRing): they stay alive
// until the profile is destroyed or the binding ends (msv_profile_bind_stream flushes first), or
// forever (shared_stream).
static bool lazy_stream(const msv_profile* p, hipStream_t st) {
    return st == p->stream || st == p->stream2 || (p->bound && st == p->bound) || (p->shared && st == p->shared);
}

// Device address of a page-locked host destination the kernels can write directly (nullptr for
// pageable memory).  Host paths then need no score D2H: the kernels' stores cross PCIe as they are
// made (a few MB of posted writes spread over the launch), and the end-of-kernel system-scope
// release makes them visible before the completion the host waits on.  (A staged D2H of the scores
// was dispatched as a blit KERNEL when queued behind the next call's launch, and starved there: the
// persistent MSV grid holds every CU -- profiles/r02_host_pipeline_timeline.txt.)
// (The same alias lets a kernel READ page-locked residues in place: see msv_score_batch.)
template <typename T>
static T* mapped_host(T* host) {
    hipPointerAttribute_t at{};
    void* h = const_cast<void*>(static_cast<const void*>(host));
    if (hipPointerGetAttributes(&at, h) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory is not an error here
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost) return nullptr;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<T*>(d);
}

// The status of a kernel's latched error bits (msv_kernel.h kErr*), most specific first.
static msv_status err_status(uint32_t err) {
    if (err & msvk::kErrBadOrder) return MSV_ERR_INVALID_ARGUMENT;  // an order entry outside the batch
    if (err & msvk::kErrBadResidue) return MSV_ERR_BAD_RESIDUE;
    if (err & msvk::kErrTooLong) return MSV_ERR_SEQUENCE_TOO_LONG;
    return MSV_OK;
}

// Whether a batch whose scores went straight to host memory had an error: a bad residue leaves +inf,
// a too-long sequence or a bad order entry NaN (msv_kernel.hip); valid scores are finite or -inf.  The
// classification of a positive answer comes from the kernel's error bits (err_status), since a NaN can
// also come out of a bad residue's +inf meeting a -inf.
static msv_status scan_scores(const float* scores, uint64_t n) {
    bool inf = false, nan = false;
    for (uint64_t i = 0; i < n; ++i) {
        const float x = scores[i];
        inf |= x == std::numeric_limits<float>::infinity();
        nan |= x != x;
    }
    if (inf) return MSV_ERR_BAD_RESIDUE;
    if (nan) return MSV_ERR_SEQUENCE_TOO_LONG;
    return MSV_OK;
}

// Lays the MSV table out for variant v and uploads it:
// [row r][chunk c][lane gl] float4 = e[r][gl*S + 4c + 1 .. +4]; states beyond LENG are -inf
// (never win a max); row 20 is the +inf poison row for codes >= 20.
// Split variants (v->sa > 0, G = 32/64, lane gl owns states gl*S + 1 .. gl*S + S as usual): an A table
// [20 rows][SA/4][G] float4 (the lane's first SA states, staged in LDS) followed by a B table
// [21 rows][G][HBP] float2 (its last S - SA states as HB = (S-SA)/2 halves padded to HBP = even,
// lane-contiguous so a lane reads them as HBP/2 float4 loads from L2; row 20 = poison).
static msv_status install_plan(msv_profile* p, const msvk::Variant* v, Plan& plan) {
    const uint32_t model_length = p->model_length, R = model_length - 1;
    const int G = v->G, S = v->S, C4 = S / 4;
    const float ninf = -std::numeric_limits<float>::infinity();
    const float pinf = std::numeric_limits<float>::infinity();
    std::vector<float> tab;
    // one [rows][chunks][G] block of `width`-float chunks whose lane gl, chunk c, slot q holds state
    // first + gl*span + width*c + q
    auto block = [&](int rows, int chunks, uint32_t first, int span, int width) {
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < chunks; ++c)
                for (int gl = 0; gl < G; ++gl)
                    for (int q = 0; q < width; ++q) {
                        const uint32_t j = first + static_cast<uint32_t>(gl * span + width * c + q);  // state 1..
                        float val;
                        if (r == msvk::kPoisonRow) val = pinf;
                        else val = (j <= R) ? p->emission_scores[static_cast<size_t>(r) * model_length + j] : ninf;
                        tab.push_back(val);
                    }
    };
    if (v->sa > 0) {
        block(msvk::kAminoAcids, v->sa / 4, 1, S, 4);
        // B table [21 rows][G][HBP] float2, lane-contiguous (each lane reads HBP/2 float4), HBP = the
        // lane's HB = (S - SA)/2 halves rounded up to even (the pad half is -inf and never read)
        const int HB = (S - v->sa) / 2, HBP = (HB + 1) & ~1;
        for (int r = 0; r < msvk::kTableRows; ++r)
            for (int gl = 0; gl < G; ++gl)
                for (int h = 0; h < HBP; ++h)
                    for (int q = 0; q < 2; ++q) {
                        const uint32_t j = static_cast<uint32_t>(v->sa + 1 + gl * S + 2 * h + q);  // state 1..
                        float val;
                        if (r == msvk::kPoisonRow) val = pinf;
                        else if (h < HB && j <= R) val = p->emission_scores[static_cast<size_t>(r) * model_length + j];
                        else val = ninf;
                        tab.push_back(val);
                    }
    } else {
        block(msvk::kTableRows, C4, 1, S, 4);
    }
    float4* d = nullptr;
    MSV_HIP(hipMalloc(reinterpret_cast<void**>(&d), tab.size() * sizeof(float)));
    hipError_t e = hipMemcpy(d, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return hip_status(e);
    }
    if (plan.d_etab) {  // may be read by an in-flight launch on any stream the caller used
        (void)hipDeviceSynchronize();
        (void)hipFree(plan.d_etab);
    }
    plan.d_etab = d;
    plan.v = v;
    hipDeviceProp_t prop;
    MSV_HIP(hipGetDeviceProperties(&prop, p->device));
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(v->fn), v->waves * 64, 0);
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    plan.blocks = prop.multiProcessorCount * per_cu;
    plan.groups_per_block = v->waves * (64 / G) * v->streams;
    return MSV_OK;
}

static void drop_plan(Plan& plan) {
    if (plan.d_etab) {  // may be read by an in-flight launch
        (void)hipDeviceSynchronize();
        (void)hipFree(plan.d_etab);
    }
    plan = Plan{};
}

// The cooperative plan (msv_coop.hip) for batches of at most one workgroup per CU: one sequence per
// workgroup, its row spread over 4 waves (one per SIMD) with halo states and a speculated B.  Installed
// when a compiled CoopVariant covers the model (the whole table staged in LDS up to 1464 states, the
// split table -- each lane's last 2-4 states read from L2 -- up to 2480) and
// tr_E_C == tr_E_J (the reference's nu = 2, MSV_HMM.cpp:49-53), and never under a forced variant.
// The smallest cooperative variant covering `states`, or nullptr.
static const msvk::CoopVariant* pick_coop_variant(uint32_t states) {
    int count = 0;
    const msvk::CoopVariant* all = msvk::coop_variants(&count);
    const msvk::CoopVariant* cv = nullptr;
    for (int i = 0; i < count; ++i)
        if (static_cast<uint32_t>(all[i].states()) >= states && (!cv || all[i].S < cv->S)) cv = &all[i];
    return cv;
}

// Lays p's table out for cooperative variant cv into `plan` (d_etab, cv).
static msv_status install_coop_table(msv_profile* p, const msvk::CoopVariant* cv, Plan& plan) {
    const uint32_t R = p->model_length - 1;
    // [21 rows][waves][SA/2 chunks][64 lanes] float2 (staged in LDS): wave w, lane l, chunk h, slot q holds
    // global state w * (64 S - halo) - halo + l S + 2h + q + 1; split variants (SA < S) append
    // [21 rows][waves][64 lanes][S - SA] floats for the lane's states SA .. S-1 (read from L2 per row).
    // States outside 1..LENG are -inf; row 20 is the +inf poison row.
    const int W = cv->waves, S = cv->S, SA = cv->sa, H = SA / 2, SB = S - SA;
    const float ninf = -std::numeric_limits<float>::infinity();
    const float pinf = std::numeric_limits<float>::infinity();
    auto value = [&](int r, int w, int l, int k) {
        const int64_t j = static_cast<int64_t>(w) * (64 * S - cv->halo) - cv->halo + l * S + k + 1;
        if (r == msvk::kPoisonRow) return pinf;
        return (j >= 1 && j <= R) ? p->emission_scores[static_cast<size_t>(r) * p->model_length + j] : ninf;
    };
    std::vector<float> tab;
    tab.reserve(static_cast<size_t>(msvk::kTableRows) * W * 64 * S);
    for (int r = 0; r < msvk::kTableRows; ++r)
        for (int w = 0; w < W; ++w)
            for (int h = 0; h < H; ++h)
                for (int l = 0; l < 64; ++l)
                    for (int q = 0; q < 2; ++q) tab.push_back(value(r, w, l, 2 * h + q));
    for (int r = 0; r < msvk::kTableRows && SB > 0; ++r)
        for (int w = 0; w < W; ++w)
            for (int l = 0; l < 64; ++l)
                for (int i = 0; i < SB; ++i) tab.push_back(value(r, w, l, SA + i));
    float4* d = nullptr;
    MSV_HIP(hipMalloc(reinterpret_cast<void**>(&d), tab.size() * sizeof(float)));
    hipError_t e = hipMemcpy(d, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return hip_status(e);
    }
    drop_plan(plan);
    plan.d_etab = d;
    plan.cv = cv;
    plan.groups_per_block = 1;
    return MSV_OK;
}

static msv_status install_coop(msv_profile* p) {
    drop_plan(p->coop);
    p->coop_max_n = 0;
    if (p->force || std::memcmp(&p->tr_E_C, &p->tr_E_J, sizeof(float)) != 0) return MSV_OK;
    const msvk::CoopVariant* cv = pick_coop_variant(p->model_length - 1);
    if (!cv) return MSV_OK;
    const msv_status st = install_coop_table(p, cv, p->coop);
    if (st != MSV_OK) return st;
    int cus = 0, per_cu = 0;
    MSV_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->device));
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cv->fn, cv->waves * 64, 0);
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    p->coop.blocks = cus * per_cu;
    // Up to where it beats the plan the batch would otherwise take (tools/coop_sweep.py,
    // profiles/r03_coop_sweep.jsonl; L U[300,500], kernel ms coop / other): 1400.hmm 512 seqs 0.106 /
    // 0.191, 1024 0.144 / 0.194, 2048 0.272 / 0.198; 1001.hmm 512 0.147 / 0.153; 1901.hmm 1024 0.243 /
    // 0.264; 2405.hmm (L ~2000) 1024 1.19 / 1.35; 400.hmm (S = 2, 768 workgroups) 512 0.037 / 0.105, 1024
    // 0.113 / 0.107; 100.hmm (no latency plan) 256 0.056 / 0.074, 512 0.071 / 0.074, 1024 0.099 / 0.074.
    // So two rounds of the grid for S >= 4, one for S = 2, half of one without a latency plan.
    const double rounds = (cv->S >= 4 ? 2.0 : 1.0) * (p->lat.v ? 1.0 : 0.5);
    p->coop_max_n = static_cast<uint64_t>(rounds * p->coop.blocks);
    return MSV_OK;
}

// Mid plan (G = 32, two sequences per wave) for G = 16 profiles with S >= 40 (~600-1536 states), taken
// by batches between the latency plan's range and about one round of the main grid.  There a 16-lane
// launch runs one partial round of 400-row sequences at ~2-3 waves per SIMD (latency-bound: ~4 ns per
// instruction per wave), and a 64-lane one needs 2-3 rounds; the 32-lane rows are half as long as the
// 16-lane ones at twice the waves.  1400.hmm x U[300,500]: 9000 sequences 0.388 ms against 0.458
// (latency plan) / 0.527 (main), 12000 0.464 vs 0.536 (main); 600.hmm x 6000 0.151 vs 0.245 (latency)
// / 0.175 (main); 900.hmm x 9000 0.299 vs 0.353 / 0.367 (profiles/r02_mid_plans.jsonl).
//  * upper end: 0.9 of one round of the main grid, and for S < 64 at most 10,752 sequences (3/4 of the
//    16,384 at which 16-lane launches fill 4 waves per SIMD: 800.hmm x 12000 ran 0.326 mid vs 0.291
//    main, while 1400.hmm x 12000 0.464 vs 0.536);
//  * lower end (the latency plan's new limit): where the 64-lane row stops being much shorter than the
//    32-lane one -- 15000 x (mid row / latency row - 1) sequences, within 1.5 rounds of the latency
//    grid: 1400.hmm (136 vs 96 VALU) ~6,100 (x 6000: 0.302 latency vs 0.306 mid), 600.hmm (76 vs 66)
//    2,270 (x 6000: mid 38% faster), 800.hmm (96 vs 76) 3,950 (x 6000: mid 8% faster).
// 500.hmm (S = 32) measured no consistent gain (the 32-lane plan won at some sizes and lost 10-15% at
// others) and keeps two plans.
static msv_status install_mid(msv_profile* p) {
    const msvk::Variant* mv = pick_mid_variant(p->model_length - 1);
    if (!mv || !p->lat.v || p->main.v->G != 16 || p->main.v->S < 40) return MSV_OK;
    const uint64_t lat_cap = static_cast<uint64_t>(p->lat.blocks) * p->lat.groups_per_block;
    const uint64_t main_cap = static_cast<uint64_t>(p->main.blocks) * p->main.groups_per_block;
    const double mid_row = 2.5 * mv->S + 26.0;
    const double lat_row = 2.5 * p->lat.v->S + 36.0 + (p->lat.v->sa ? 2.0 : 0.0);
    const uint64_t lat_by_rows = static_cast<uint64_t>(std::max(0.0, 15000.0 * (mid_row / lat_row - 1.0)));
    const uint64_t lat_max = std::min({p->lat_max_n, lat_cap * 3 / 2, lat_by_rows});
    const uint64_t mid_max = std::min<uint64_t>(main_cap * 9 / 10, p->main.v->S >= 64 ? ~0ull : 10752);
    if (mid_max <= lat_max) return MSV_OK;
    msv_status s = install_plan(p, mv, p->mid);
    if (s != MSV_OK) return s;
    p->lat_max_n = lat_max;
    p->mid_max_n = mid_max;
    return MSV_OK;
}

// Main plan for `v`; unless forced, the latency plan (its own table layout) unless it would be the same
// kernel, and a mid plan (install_mid; or, when the main plan has 4-lane groups, the 16-lane plan for
// batches that leave the SIMDs part-empty).
static msv_status install_variant_plans(msv_profile* p, const msvk::Variant* main_v) {
    msv_status s = install_plan(p, main_v, p->main);
    if (s != MSV_OK) return s;
    const uint32_t states = p->model_length - 1;
    // the 16+-lane plan the latency plan is weighed against, and the plan of batches below one round of
    // the grid: the main plan itself unless it is narrow (4 lanes) or a whole-row-ring variant
    const msvk::Variant* v =
        (main_v->G < 16 || whole_row_ring(*main_v)) && !p->force ? pick_variant(states, false) : main_v;
    const msvk::Variant* lv = p->force ? nullptr : pick_latency_variant(states);
    // Worth it only when the 64-lane row is much shorter than the main row (per-row issue cost,
    // as variant_cost): 1400.hmm 246 vs 96 -> 0.23 vs 0.62 ms at 1024 sequences, 0.37 vs 0.64 at 8192,
    // even at 16384; 1901.hmm 176 vs 123 -> 0.97 vs 1.29 ms at 3 sequences, 1.99 vs 2.89 at 2048;
    // 100.hmm 46 vs 46 -> slower at every size (tools/tune.py, profiles/r01_latency_plan.jsonl,
    // r02_latency_plans.jsonl).
    const double main_row = 2.5 * v->S + 26.0, lat_row = lv ? 2.5 * lv->S + 36.0 + (lv->sa ? 2.0 : 0.0) : 0.0;
    const double ratio = lv ? main_row / lat_row : 0.0;
    drop_plan(p->mid);
    p->mid_max_n = 0;
    if (v != main_v) {
        // Narrow main plan: the 16-lane plan while it would not fill the SIMDs -- 3.5 of its waves per
        // SIMD, where a 16-lane launch turns issue-bound (100.hmm: 14,336 sequences on 256 CUs; the
        // crossover measured between 10k and 20k, profiles/r02_small_profiles.jsonl).  Whole-row-ring
        // main plan: the PF-2 variant up to 3/4 of that (10,752).
        int cus = 0;
        MSV_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->device));
        s = install_plan(p, v, p->mid);
        if (s != MSV_OK) return s;
        const double fill = main_v->G < 16 ? 3.5 : 2.625;
        p->mid_max_n = static_cast<uint64_t>(fill * 4 * cus * (64 / v->G));
    }
    if (!lv || lv == v || ratio < 1.3) {
        drop_plan(p->lat);
        p->lat_max_n = 0;
        return MSV_OK;
    }
    p->lat_max_n = static_cast<uint64_t>(std::min(12288.0, 4096.0 * ratio));
    s = install_plan(p, lv, p->lat);
    if (s != MSV_OK) return s;
    if (p->mid.v) {
        p->lat_max_n = std::min(p->lat_max_n, p->mid_max_n);
        return MSV_OK;
    }
    return install_mid(p);
}

// The main / mid / latency plans, then the cooperative plan in front of them (it needs to know whether a
// latency plan exists: install_coop).
static msv_status install_variant(msv_profile* p, const msvk::Variant* main_v) {
    const msv_status s = install_variant_plans(p, main_v);
    if (s != MSV_OK) return s;
    return install_coop(p);
}

// Pieces of a host batch for msv_score_batch's copy/compute pipeline: cut[k] .. cut[k+1] is piece
// k's sequence range.  Each piece addresses < kChunkBytes residues and < 2^32 - 2^24 sequences (one
// launch each).  Batches below kPipelineMin residues are one piece; larger ones start at 1/first_den
// of the batch (at least 1M residues) and grow `growth`-fold, a short remainder joining the last piece.
static std::vector<uint64_t> plan_pieces(const uint64_t* offsets, uint64_t n, uint64_t total, uint32_t first_den,
                                         uint32_t growth) {
    constexpr uint64_t kMaxSeqs = (1ull << 32) - (1ull << 24) - 1;
    std::vector<uint64_t> cut{0};
    uint64_t want = (total < kPipelineMin || first_den == 0) ? kChunkBytes
                                                             : std::max<uint64_t>(1ull << 20, total / first_den);
    uint64_t first = 0;
    while (first < n) {
        const uint64_t base = offsets[first];
        auto end_of = [&](uint64_t budget) {  // last sequence index with offsets[last] - base <= budget
            const uint64_t* it = std::upper_bound(offsets + first + 1, offsets + n + 1, base + budget);
            return static_cast<uint64_t>(it - offsets) - 1;
        };
        uint64_t last = std::max(end_of(std::min(want, kChunkBytes - 1)), first + 1);  // >= one sequence
        last = std::min(last, first + kMaxSeqs);
        // a remainder shorter than this piece joins it (half the next piece at the default growth of 2),
        // if the chunk limit allows
        const uint64_t rest = offsets[n] - offsets[last];
        if (last < n && rest < want && offsets[n] - base < kChunkBytes && n - first <= kMaxSeqs) last = n;
        cut.push_back(last);
        first = last;
        want = std::min(kChunkBytes, std::max<uint32_t>(growth, 1) * want);
    }
    return cut;
}

extern "C" {

msv_status msv_device_count(int* count) {
    if (!count) return MSV_ERR_INVALID_ARGUMENT;
    *count = 0;
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return MSV_ERR_NO_DEVICE;
    }
    return MSV_OK;
}

void msv_profile_destroy(msv_profile* p) {
    if (!p) return;
    DeviceGuard g(p->device);
    // work still queued on any stream (an unwaited msv_score_batch_async call, a device call on the
    // caller's stream) may use the buffers and pinned staging freed below
    (void)hipDeviceSynchronize();
    (void)hipFree(p->main.d_etab);
    (void)hipFree(p->lat.d_etab);
    (void)hipFree(p->mid.d_etab);
    (void)hipFree(p->fused.d_etab);
    (void)hipFree(p->coop.d_etab);
    (void)hipFree(p->coop_fused.d_etab);
    (void)hipFree(p->d_lentab);
    (void)hipFree(p->d_words);
    (void)hipFree(p->d_hist);
    (void)hipFree(p->d_dummy);
    (void)hipFree(p->d_res);
    (void)hipFree(p->d_off);
    (void)hipFree(p->d_scores);
    (void)hipFree(p->d_order);
    if (p->h_off) (void)hipHostFree(p->h_off);
    if (p->h_sc) (void)hipHostFree(p->h_sc);
    if (p->done) (void)hipEventDestroy(p->done);
    for (hipEvent_t e : p->events) (void)hipEventDestroy(e);
    p->kernels.destroy();
    p->orders.destroy();
    for (auto& a : p->async) {
        if (a.copied) (void)hipEventDestroy(a.copied);
        if (a.off_copied) (void)hipEventDestroy(a.off_copied);
        if (a.done) (void)hipEventDestroy(a.done);
        (void)hipFree(a.d_res);
        (void)hipFree(a.d_off);
        (void)hipFree(a.d_sc);
        (void)hipFree(a.d_ord);
        if (a.h_off) (void)hipHostFree(a.h_off);
        if (a.h_err) (void)hipHostFree(a.h_err);
    }
    if (p->stream) (void)hipStreamDestroy(p->stream);
    if (p->stream2) (void)hipStreamDestroy(p->stream2);
    if (p->copy_stream) (void)hipStreamDestroy(p->copy_stream);
    if (p->offsets_stream) (void)hipStreamDestroy(p->offsets_stream);
    delete p;
}

msv_status msv_profile_reserve_length(msv_profile* p, uint64_t max_length) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    if (max_length >= (1ull << 31)) return MSV_ERR_SEQUENCE_TOO_LONG;
    const uint32_t need = static_cast<uint32_t>(max_length) + 1;
    if (need <= p->lentab_n) return MSV_OK;
    DeviceGuard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    const uint32_t n = std::max(need, p->lentab_n * 2);
    const std::vector<float2> host = host_length_table(n);
    float2* d = nullptr;
    MSV_HIP(hipMalloc(reinterpret_cast<void**>(&d), n * sizeof(float2)));
    hipError_t e = hipMemcpy(d, host.data(), n * sizeof(float2), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return hip_status(e);
    }
    // the old table may still be read by an in-flight launch on any stream the caller used
    if (p->d_lentab) {
        (void)hipDeviceSynchronize();
        (void)hipFree(p->d_lentab);
    }
    p->d_lentab = d;
    p->lentab_n = n;
    return MSV_OK;
}

msv_status msv_profile_create(int device, const float* emission_scores, uint32_t model_length, float tr_B_Mk,
                              float tr_E_C, float tr_E_J, msv_profile** out) {
    if (!emission_scores || !out || model_length < 2) return MSV_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return MSV_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return MSV_ERR_NO_DEVICE;
    const uint32_t R = model_length - 1;  // real match states (MSV_HMM.cpp:285)
    const msvk::Variant* v = pick_variant(R, true, true);
    if (!v) return MSV_ERR_UNSUPPORTED_MODEL;

    DeviceGuard g(device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    auto* p = new (std::nothrow) msv_profile;
    if (!p) return MSV_ERR_OUT_OF_MEMORY;
    p->device = device;
    p->model_length = model_length;
    p->tr_B_Mk = tr_B_Mk;
    p->tr_E_C = tr_E_C;
    p->tr_E_J = tr_E_J;

    p->emission_scores.assign(emission_scores, emission_scores + static_cast<size_t>(20) * model_length);
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking)) != hipSuccess) {
        msv_profile_destroy(p);
        return hip_status(e);
    }
    // every launch slot's event up front: created lazily, the first kLaunchSlots launches of a fresh
    // profile each paid an event creation (~10 us; 24 of them in one fused grid call)
    for (LaunchRing* ring : {&p->kernels, &p->orders})
        if ((e = ring->create_events()) != hipSuccess) {
            msv_profile_destroy(p);
            return hip_status(e);
        }
    if ((e = hipMalloc(reinterpret_cast<void**>(&p->d_words), kWords * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMemset(p->d_words, 0, kWords * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&p->d_dummy), 64)) != hipSuccess ||
        (e = hipMemset(p->d_dummy, 0, 64)) != hipSuccess) {
        msv_profile_destroy(p);
        return hip_status(e);
    }
    msv_status s = install_variant(p, v);
    if (s != MSV_OK) {
        msv_profile_destroy(p);
        return s;
    }
    s = msv_profile_reserve_length(p, kDefaultMaxLength - 1);
    if (s != MSV_OK) {
        msv_profile_destroy(p);
        return s;
    }
    *out = p;
    return MSV_OK;
}

int msv_variant_count(void) {
    int count = 0;
    (void)msvk::variants(&count);
    return count;
}

const char* msv_variant_name(int i) {
    int count = 0;
    const msvk::Variant* all = msvk::variants(&count);
    return (i >= 0 && i < count) ? all[i].name : nullptr;
}

msv_status msv_profile_set_variant(msv_profile* p, const char* name) {
    if (!p || !name) return MSV_ERR_INVALID_ARGUMENT;
    int count = 0;
    const msvk::Variant* all = msvk::variants(&count);
    for (int i = 0; i < count; ++i) {
        if (std::strcmp(all[i].name, name) != 0) continue;
        if (static_cast<uint32_t>(all[i].G * all[i].S) < p->model_length - 1) return MSV_ERR_UNSUPPORTED_MODEL;
        DeviceGuard g(p->device);
        if (!g.ok) return MSV_ERR_NO_DEVICE;
        p->force = true;  // a forced variant runs every batch (tests, tools/tune.py)
        return install_variant(p, &all[i]);
    }
    return MSV_ERR_INVALID_ARGUMENT;
}

// Diagnostics, deliberately not in msv.h: a device buffer of msvk::kStampWords (6) uint64 per wave of the
// persistent grid that receives {start, end (s_memrealtime, 100 MHz), rows issued, xcc<<32|block, shader
// clock start, end (s_memtime)} for every wave of subsequent launches (tools/wave_timeline.py, bench.py's
// clock_GHz).  nullptr switches it off.
msv_status msv_debug_set_stamps(msv_profile* p, uint64_t* d_stamps) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    p->d_stamps = d_stamps;
    p->stamp_clock = false;
    return MSV_OK;
}

// Diagnostics (bench.py roofline.clock_GHz), not in msv.h: subsequent launches of plans that have a CLOCK twin
// (msv_kernel_impl.h clock_fn) run it and write msvk::kStampWords (6) uint64 per wave -- the 4 stamps above plus
// shader-clock ticks (s_memtime) at the wave's start and end; launches of other plans write nothing.
// nullptr switches it off.
msv_status msv_debug_set_clock_stamps(msv_profile* p, uint64_t* d_stamps) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    p->d_stamps = d_stamps;
    p->stamp_clock = d_stamps != nullptr;
    return MSV_OK;
}

// Diagnostics (not in msv.h): the host pipeline's piece plan -- the first piece is 1/first_den of the
// batch, each next one `growth` times larger; first_den = 0 scores the batch as one piece; pieces
// alternate over `streams` (1 or 2) compute streams.
msv_status msv_debug_set_pipeline(msv_profile* p, uint32_t first_den, uint32_t growth, uint32_t streams) {
    if (!p || growth == 0 || streams < 1 || streams > 2) return MSV_ERR_INVALID_ARGUMENT;
    p->pipe_first_den = first_den;
    p->pipe_growth = growth;
    p->pipe_streams = streams;
    return MSV_OK;
}

// Diagnostics (not in msv.h): the profile's next MSV launch updates `start` / `stop` (hipEvent_t, created
// with timing) with its own start and end through hipExtLaunchKernel -- the kernel duration without the
// two marker packets (~4 us each on the stream) that event records around the launch would add.
msv_status msv_debug_time_next_launch(msv_profile* p, void* start, void* stop) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    p->time_start = static_cast<hipEvent_t>(start);
    p->time_stop = static_cast<hipEvent_t>(stop);
    return MSV_OK;
}

// Diagnostics (not in msv.h): batches up to n sequences take the cooperative plan (tools/coop_sweep.py;
// 0 turns it off).  Returns MSV_ERR_UNSUPPORTED_MODEL when the profile has no cooperative plan.
msv_status msv_debug_set_coop_max_n(msv_profile* p, uint64_t n) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    if (!p->coop.cv) return MSV_ERR_UNSUPPORTED_MODEL;
    p->coop_max_n = n;
    return MSV_OK;
}

// Diagnostics (not in msv.h): how msv_score_batch treats page-locked residues.  on: 0 = copied (pipeline),
// 1 = read in place, 2 = read in place but without the wide-block twins (A/B of the 64-byte superblock
// requests against the 16-byte block requests).
msv_status msv_debug_set_zero_copy(msv_profile* p, int on) {
    if (!p || on < 0 || on > 2) return MSV_ERR_INVALID_ARGUMENT;
    p->zero_copy = on != 0;
    p->zc_wide = on != 2;
    return MSV_OK;
}

int msv_debug_grid_waves(const msv_profile* p) {
    if (!p) return 0;
    const int lat = p->lat.v ? p->lat.blocks * p->lat.v->waves : 0;
    const int mid = p->mid.v ? p->mid.blocks * p->mid.v->waves : 0;
    return std::max({p->main.blocks * p->main.v->waves, lat, mid});  // the stamps buffer must fit every plan
}

msv_status msv_profile_create_from_hmm(int device, const msv_hmm* hmm, msv_profile** out) {
    if (!hmm || !out) return MSV_ERR_INVALID_ARGUMENT;
    const size_t M = msv_hmm_model_length(hmm);
    std::vector<float> es(M * 20);
    float b, c, j;
    msv_status s = msv_hmm_msv_scores(hmm, es.data(), &b, &c, &j);
    if (s != MSV_OK) return s;
    return msv_profile_create(device, es.data(), static_cast<uint32_t>(M), b, c, j, out);
}

msv_status msv_profile_describe(const msv_profile* p, msv_kernel_info* out) {
    if (!p || !out) return MSV_ERR_INVALID_ARGUMENT;
    std::memset(out, 0, sizeof(*out));
    out->model_length = p->model_length;
    const msvk::Variant* v = p->main.v;
    out->lanes_per_group = static_cast<uint32_t>(v->G);
    out->states_per_lane = static_cast<uint32_t>(v->S);
    out->waves_per_block = static_cast<uint32_t>(v->waves);
    out->lds_rows = static_cast<uint32_t>(v->lds_rows);
    out->lds_bytes = static_cast<uint32_t>(v->lds_rows * v->G * (v->sa ? v->sa : v->S) * 4);
    out->blocks = static_cast<uint32_t>(p->main.blocks);
    out->max_length = p->lentab_n ? p->lentab_n - 1 : 0;
    out->device = p->device;
    std::snprintf(out->variant, sizeof(out->variant), "%s", v->name);
    // the small-batch (latency) plan, if this profile has one
    if (p->lat.v) {
        std::snprintf(out->latency_variant, sizeof(out->latency_variant), "%s", p->lat.v->name);
        out->latency_blocks = static_cast<uint32_t>(p->lat.blocks);
        out->latency_max_n = p->lat_max_n;
    }
    if (p->coop.cv) {
        std::snprintf(out->coop_variant, sizeof(out->coop_variant), "%s", p->coop.cv->name);
        out->coop_blocks = static_cast<uint32_t>(p->coop.blocks);
        out->coop_max_n = p->coop_max_n;
    }
    if (p->mid.v) {
        std::snprintf(out->mid_variant, sizeof(out->mid_variant), "%s", p->mid.v->name);
        out->mid_blocks = static_cast<uint32_t>(p->mid.blocks);
        out->mid_max_n = p->mid_max_n;
    }
    return MSV_OK;
}

// The plan a launch of n sequences takes: latency (n <= lat_max_n), mid (n <= mid_max_n), else main.
static const Plan& select_plan(const msv_profile* p, uint64_t n, bool latency_ok, bool host_residues = false) {
    if (!latency_ok) return p->main;
    // (not for residues read in place over PCIe: its 16-row residue blocks would wait on each one)
    if (p->coop.cv && n <= p->coop_max_n && !host_residues) return p->coop;
    if (p->lat.v && n <= p->lat_max_n) return p->lat;
    if (p->mid.v && n <= p->mid_max_n) return p->mid;
    return p->main;
}

// A batch that takes the cooperative plan with at most one sequence per workgroup needs no dequeue order
// (every workgroup scores one sequence whatever the order): the host paths then skip the sort launch.
static bool order_needless(const msv_profile* p, uint64_t n, bool host_residues) {
    const Plan& plan = select_plan(p, n, true, host_residues);
    return plan.cv && n <= static_cast<uint64_t>(plan.blocks);
}

const char* msv_profile_variant_for(const msv_profile* p, uint64_t n) {
    if (!p || !p->main.v) return "";
    const Plan& plan = select_plan(p, n, true);
    return plan.cv ? plan.cv->name : plan.v->name;
}

// One MSV launch.  `latency_ok`: a batch of few sequences may take the latency plan (not for the
// pieces of a host pipeline, whose kernels must share the CUs with the next piece's).
static msv_status launch_batch(msv_profile* p, const uint8_t* d_residues, uint64_t residues_len,
                               const uint64_t* d_offsets, uint64_t n, const uint32_t* d_order, float* d_scores,
                               void* stream, bool latency_ok, uint32_t* d_errors = nullptr,
                               bool host_residues = false) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    if (n == 0) return MSV_OK;
    if (!d_offsets || !d_scores || (residues_len && !d_residues)) return MSV_ERR_INVALID_ARGUMENT;
    if (residues_len >= (1ull << 32) || n >= (1ull << 32) - (1ull << 24)) return MSV_ERR_INVALID_ARGUMENT;
    DeviceGuard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : p->stream;

    msvk::KernelArgs a{};
    // Small batches take the latency plan: with fewer sequences than ~4 per SIMD the launch lasts
    // one sequence's rows, and a 64-lane row is far shorter than a 16-lane one.  Mid-size ones (less
    // than one round of the main grid) take the 32-lane plan where there is one (install_variant).
    const Plan& plan = select_plan(p, n, latency_ok, host_residues);
    a.etab = plan.d_etab;
    a.residues = residues_len ? d_residues : p->d_dummy;
    a.offsets = d_offsets;
    a.order = d_order;
    a.lentab = p->d_lentab;
    a.scores = d_scores;
    a.n = n;
    a.lentab_n = p->lentab_n;
    a.tr_B_Mk = p->tr_B_Mk;
    a.tr_E_C = p->tr_E_C;
    a.tr_E_J = p->tr_E_J;
    a.stamps = p->d_stamps;
    const bool clock = p->stamp_clock && !host_residues;
    if (p->stamp_clock && (plan.cv || !plan.v->clock_fn || host_residues)) a.stamps = nullptr;  // no CLOCK twin

    const uint64_t want = (n + plan.groups_per_block - 1) / plan.groups_per_block;
    const int blocks = static_cast<int>(std::min<uint64_t>(static_cast<uint64_t>(plan.blocks), want));
    if (plan.cv) {  // the cooperative plan: a workgroup per sequence, no dequeue counter
        a.errors = d_errors ? d_errors : p->d_words + kErrWord;
        hipEvent_t t0 = p->time_start, t1 = p->time_stop;
        p->time_start = p->time_stop = nullptr;
        void* params[] = {&a};
        const dim3 block(static_cast<uint32_t>(plan.cv->waves * 64));
        MSV_HIP(t0 || t1 ? hipExtLaunchKernel(plan.cv->fn, dim3(blocks), block, params, 0, st, t0, t1, 0)
                         : hipLaunchKernel(plan.cv->fn, dim3(blocks), block, params, 0, st));
        return MSV_OK;
    }
    // A slot's counters (next index, waves left) are zero between launches: zeroed at creation and
    // put back by the last wave of every launch (msv_kernel.hip).  A failed launch may leave them
    // dirty, so the slot's next launch resets them explicitly.
    int k = 0;
    MSV_HIP(p->kernels.acquire(st, &k));
    a.counter = p->d_words + 2 * k;
    a.errors = d_errors ? d_errors : p->d_words + kErrWord;
    if (p->kernels.dirty[k]) MSV_HIP(hipMemsetAsync(a.counter, 0, 2 * sizeof(uint32_t), st));
    p->kernels.dirty[k] = true;
    hipEvent_t t0 = p->time_start, t1 = p->time_stop;
    p->time_start = p->time_stop = nullptr;
    // the twin of a residue-block variant (rows of <= 40 states) reads 4-byte superblock words, clamped
    // to the buffer only from 4 bytes up: it takes buffers of at least 64 bytes
    const bool wide = plan.v->S <= 40;  // (twins of rows > 40 states prefetch two rows; see zc_fn)
    const bool twin = host_residues && (!wide || (p->zc_wide && residues_len >= 64));
    MSV_HIP(msvk::launch_variant(*plan.v, dim3(blocks), a, st, t0, t1, twin, clock));
    p->kernels.dirty[k] = false;
    MSV_HIP(p->kernels.release(k, st, lazy_stream(p, st)));
    return MSV_OK;
}

msv_status msv_score_batch_device(msv_profile* p, const uint8_t* d_residues, uint64_t residues_len,
                                  const uint64_t* d_offsets, uint64_t n, const uint32_t* d_order, float* d_scores,
                                  void* stream) {
    return launch_batch(p, d_residues, residues_len, d_offsets, n, d_order, d_scores, stream, true);
}

// Library-internal (msv_score_batch, msv_multi.cpp): whether page-locked residues of `bytes` bytes are read
// in place (zero-copy) rather than copied -- see msv_score_batch.
__attribute__((visibility("hidden"))) bool msv_in_place_wins(const msv_profile* p, uint64_t bytes) {
    return p->model_length - 1 >= kInPlaceMinStates || bytes < kInPlaceAnyBytes;
}

// Library-internal (msv_multi.cpp): msv_score_batch_device for residues that are the device alias of
// page-locked host memory -- the launch takes the variant's zero-copy twin (msv_kernel.hip zc_fn).
__attribute__((visibility("hidden"))) msv_status msv_score_batch_host_residues(
    msv_profile* p, const uint8_t* d_residues, uint64_t residues_len, const uint64_t* d_offsets, uint64_t n,
    const uint32_t* d_order, float* d_scores, void* stream) {
    return launch_batch(p, d_residues, residues_len, d_offsets, n, d_order, d_scores, stream, true, nullptr, true);
}

msv_status msv_profile_bind_stream(msv_profile* p, void* stream) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (st == p->bound) return MSV_OK;
    DeviceGuard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    if (p->bound) {  // the old stream loses its guarantee: record what is still pending on it
        MSV_HIP(p->kernels.flush(p->bound));
        MSV_HIP(p->orders.flush(p->bound));
    }
    p->bound = st;
    return MSV_OK;
}

// Synchronises `st`, then reads, clears and reports error word `word` of the profile.
static msv_status check_word(msv_profile* p, hipStream_t st, int word) {
    uint32_t err = 0;
    MSV_HIP(hipMemcpyAsync(&err, p->d_words + word, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    MSV_HIP(hipStreamSynchronize(st));
    if (err) MSV_HIP(hipMemsetAsync(p->d_words + word, 0, sizeof(uint32_t), st));
    MSV_HIP(hipStreamSynchronize(st));
    return err_status(err);
}

msv_status msv_profile_check(msv_profile* p, void* stream) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    DeviceGuard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    return check_word(p, stream ? static_cast<hipStream_t>(stream) : p->stream, kErrWord);
}

msv_status msv_order_longest_first(msv_profile* p, const uint64_t* d_offsets, uint64_t n, uint32_t* d_order,
                                   void* stream) {
    if (!p || (n && (!d_offsets || !d_order))) return MSV_ERR_INVALID_ARGUMENT;
    if (n == 0) return MSV_OK;
    DeviceGuard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : p->stream;
    if (!p->d_hist) {
        MSV_HIP(hipMalloc(reinterpret_cast<void**>(&p->d_hist),
                            kLaunchSlots * msvk::kOrderScratchWords(kOrderBins) * sizeof(uint32_t)));
        p->hist_dirty.fill(true);
    }
    int k = 0;
    MSV_HIP(p->orders.acquire(st, &k));
    // [histogram | cursors | ticket] per slot; the sort leaves histogram and ticket zeroed for the slot's next use
    uint32_t* scratch = p->d_hist + static_cast<size_t>(k) * msvk::kOrderScratchWords(kOrderBins);
    if (p->hist_dirty[k])
        MSV_HIP(hipMemsetAsync(scratch, 0, msvk::kOrderScratchWords(kOrderBins) * sizeof(uint32_t), st));
    p->hist_dirty[k] = true;
    MSV_HIP(msvk::launch_order(d_offsets, n, scratch, kOrderBins, d_order, st));
    p->hist_dirty[k] = false;
    MSV_HIP(p->orders.release(k, st, lazy_stream(p, st)));
    return MSV_OK;
}

msv_status msv_host_alloc(size_t bytes, void** out) {
    if (!out) return MSV_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    MSV_HIP(hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocPortable));
    return MSV_OK;
}

msv_status msv_host_free(void* ptr) {
    if (ptr) MSV_HIP(hipHostFree(ptr));
    return MSV_OK;
}

msv_status msv_score_batch(msv_profile* p, const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                           float* scores, void* stream) {
    if (!p || (n && (!offsets || !scores))) return MSV_ERR_INVALID_ARGUMENT;
    if (n == 0) return MSV_OK;
    // Validate the CSR on the host (cheap, O(n)) and find the longest sequence.
    uint64_t maxL = 0;
    for (uint64_t s = 0; s < n; ++s) {
        if (offsets[s + 1] < offsets[s]) return MSV_ERR_INVALID_ARGUMENT;
        maxL = std::max<uint64_t>(maxL, offsets[s + 1] - offsets[s]);
    }
    if (maxL >= kChunkBytes) return MSV_ERR_SEQUENCE_TOO_LONG;
    const uint64_t total = offsets[n] - offsets[0];
    if (total && !residues) return MSV_ERR_INVALID_ARGUMENT;
    msv_status s = msv_profile_reserve_length(p, maxL);
    if (s != MSV_OK) return s;

    DeviceGuard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : p->stream;

    // Copy/compute pipeline.  The batch is cut into pieces (contiguous sequence ranges) whose
    // residue counts grow geometrically from 1/4 of the batch (x2: 2 pieces for cfg3, the best plan
    // in tools/host_pipeline_sweep.py, profiles/r02_host_pipeline_sweep.jsonl), so the first kernel
    // starts after a short copy and every later piece's H2D (copy stream) runs under the kernels of
    // the pieces before it.  All offsets go first, and every piece's longest-first order runs before
    // the first kernel (under piece 0's residue copy).  Pieces alternate between two compute
    // streams, so a piece's kernel fills the CUs that the previous piece's drain tail frees (each
    // launch has its own dequeue counter slot).  Scores and the error word come back once at the end
    // (pageable destinations would make per-piece D2H copies block the host thread that enqueues the
    // pipeline), followed by ONE synchronisation.
    // Page-locked residues are not copied at all: the kernel reads them in place over PCIe through their
    // device alias (zero-copy; L2 keeps each 128-B line for the rows that follow).  cfg3: kernel 2.98 vs
    // 2.87 ms from HBM -- 0.96 of the resident rate with no copy, against ~0.85 for the copy pipeline
    // below, whose first piece's copy and extra drain tail it saves (profiles/r02_zero_copy_probe.jsonl).
    // One launch per < 2^32-byte piece; no copy stream, no second compute stream.
    // Except for large batches of small models, whose kernel consumes residues faster than the ~25 GB/s at
    // which a kernel reads host memory: page-locked 100k x U[300,500] batches, per call in place vs copied
    // (profiles/r03_ab_in_place_vs_copied.jsonl): 100.hmm 1.60 vs 1.24 ms, 200.hmm 1.69 vs 1.46, 400.hmm
    // 1.68 vs 1.76, 600.hmm 1.75 vs 2.33, 1400.hmm 3.09 vs 3.36; 100.hmm x 20k (8 MB) 0.41 vs 0.44.
    const bool in_place_wins = msv_in_place_wins(p, total);
    const uint8_t* const zres = (total && p->zero_copy && in_place_wins) ? mapped_host(residues) : nullptr;
    const std::vector<uint64_t> cut = plan_pieces(offsets, n, total, zres ? 0 : p->pipe_first_den, p->pipe_growth);
    const size_t P = cut.size() - 1;
    // SMALL calls: the residues ride in the offsets' H2D (behind the n + 1 offsets, in u64 words), and
    // pageable scores are written by the kernel into pinned staging.  A one-sequence call was two H2D
    // and two D2H blits, the scores' D2H to pageable memory a ~25 us round trip on the host
    // (profiles/r03_reference_call_timeline.txt).
    const bool small = !zres && total <= kSmallCall && n <= kSmallCall;
    const uint64_t res_words = small ? (total + 7) / 8 : 0;
    if (!zres && !small) MSV_HIP(ensure(p->d_res, p->d_res_cap, std::max<uint64_t>(total, 1)));
    MSV_HIP(ensure(p->d_off, p->d_off_cap, n + P + res_words));
    // a page-locked destination is written by the kernels themselves (no D2H of the scores)
    float* direct = mapped_host(scores);
    const bool staged_scores = !direct && small;
    if (staged_scores) {
        if (p->h_sc_cap < n) {
            if (p->h_sc) (void)hipHostFree(p->h_sc);
            p->h_sc = nullptr;
            p->h_sc_cap = 0;
            MSV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p->h_sc), std::max<uint64_t>(n, 64) * sizeof(float),
                                  hipHostMallocDefault));
            p->h_sc_cap = std::max<uint64_t>(n, 64);
        }
        direct = mapped_host(p->h_sc);
        if (!direct) return MSV_ERR_HIP;
    }
    if (!direct) MSV_HIP(ensure(p->d_scores, p->d_scores_cap, n));
    float* const dsc = direct ? direct : p->d_scores;
    MSV_HIP(ensure(p->d_order, p->d_order_cap, n));
    if (p->h_off_cap < n + P + 8 + res_words) {  // pinned: the offsets H2D is a true async DMA (+ the error word)
        if (p->h_off) (void)hipHostFree(p->h_off);
        p->h_off = nullptr;
        p->h_off_cap = 0;
        MSV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p->h_off), (n + P + 8 + res_words) * sizeof(uint64_t),
                              hipHostMallocDefault));
        p->h_off_cap = n + P + 8 + res_words;
    }
    uint32_t* h_err = reinterpret_cast<uint32_t*>(p->h_off + n + P + res_words);
    const uint8_t* const d_small_res = reinterpret_cast<const uint8_t*>(p->d_off + n + P);  // SMALL: residues
    const bool pipe = P > 1 && !zres;
    hipStream_t cs[2] = {st, st}, cp = st;
    // On an early error return, copies reading the pinned h_off (rewritten by the next call) and
    // kernels writing the staging buffers may still be queued: drain every stream used first.
    struct Drain {
        hipStream_t* cs;
        hipStream_t* cp;
        bool armed = true;
        ~Drain() {
            if (!armed) return;
            (void)hipStreamSynchronize(cs[0]);
            (void)hipStreamSynchronize(cs[1]);
            (void)hipStreamSynchronize(*cp);
        }
    } drain{cs, &cp};
    if (pipe) {
        if (!p->stream2) MSV_HIP(hipStreamCreateWithFlags(&p->stream2, hipStreamNonBlocking));
        if (!p->copy_stream) MSV_HIP(hipStreamCreateWithFlags(&p->copy_stream, hipStreamNonBlocking));
        cs[1] = p->pipe_streams == 2 ? p->stream2 : st;
        cp = p->copy_stream;
        while (p->events.size() < P + 4) {
            hipEvent_t e = nullptr;
            MSV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice));
            p->events.push_back(e);
        }
        // fork: both helper streams start after the caller's stream's earlier work
        MSV_HIP(hipEventRecord(p->events[P + 2], st));
        MSV_HIP(hipStreamWaitEvent(cp, p->events[P + 2], 0));
        MSV_HIP(hipStreamWaitEvent(cs[1], p->events[P + 2], 0));
    }
    // 1. the residue pieces go first, in order, on the copy stream: their DMA is the critical path
    const uint64_t base0 = offsets[0];
    for (size_t k = 0; k < P; ++k) {
        const uint64_t lo = offsets[cut[k]] - base0, bytes = offsets[cut[k + 1]] - offsets[cut[k]];
        if (bytes && !zres && !small)
            MSV_HIP(hipMemcpyAsync(p->d_res + lo, residues + base0 + lo, bytes, hipMemcpyHostToDevice, cp));
        if (pipe) MSV_HIP(hipEventRecord(p->events[2 + k], cp));  // piece k's residues landed
    }
    // 2. meanwhile every piece's offsets (rebased on the piece's first residue, at h_off[cut[k] + k ..])
    //    in ONE H2D on the caller's stream, then every piece's longest-first order there, under the
    //    first residue copy (an order kernel enqueued behind a running MSV kernel would find no free
    //    VGPRs until that kernel's blocks drain, delaying the next piece's launch)
    for (size_t k = 0; k < P; ++k) {
        uint64_t* ho = p->h_off + cut[k] + k;
        const uint64_t base = offsets[cut[k]], cn = cut[k + 1] - cut[k];
        for (uint64_t i = 0; i <= cn; ++i) ho[i] = offsets[cut[k] + i] - base;
    }
    if (small && total) std::memcpy(p->h_off + n + P, residues + base0, total);
    MSV_HIP(hipMemcpyAsync(p->d_off, p->h_off, (n + P + res_words) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    const bool sort = pipe || !order_needless(p, n, zres != nullptr);
    for (size_t k = 0; k < P && sort; ++k) {
        s = msv_order_longest_first(p, p->d_off + cut[k] + k, cut[k + 1] - cut[k], p->d_order + cut[k], st);
        if (s != MSV_OK) return s;
    }
    if (pipe) {
        MSV_HIP(hipEventRecord(p->events[1], st));  // offsets and orders done
        MSV_HIP(hipStreamWaitEvent(cs[1], p->events[1], 0));
    }
    // 3. the kernels, alternating over the compute streams so that the LAST piece runs on the caller's
    //    stream (the scores' D2H then waits on no other stream), each after its piece's residues
    for (size_t k = 0; k < P; ++k) {
        const uint64_t lo = offsets[cut[k]] - base0, bytes = offsets[cut[k + 1]] - offsets[cut[k]];
        hipStream_t c = cs[(P - 1 - k) & 1];
        if (pipe) MSV_HIP(hipStreamWaitEvent(c, p->events[2 + k], 0));
        const uint8_t* src = zres ? zres + base0 + lo : (small ? d_small_res : p->d_res) + lo;
        s = launch_batch(p, bytes ? src : p->d_dummy, std::max<uint64_t>(bytes, 1), p->d_off + cut[k] + k,
                         cut[k + 1] - cut[k], sort ? p->d_order + cut[k] : nullptr, dsc + cut[k], c, !pipe,
                         p->d_words + kHostErrWord, zres && bytes);
        if (s != MSV_OK) return s;
    }
    if (pipe) {  // join the second compute stream (done before the last piece) back into the caller's
        MSV_HIP(hipEventRecord(p->events[P + 3], cs[1]));
        MSV_HIP(hipStreamWaitEvent(st, p->events[P + 3], 0));
    }
    if (direct) {
        // scores in page-locked memory: every error leaves a score that is +inf or NaN (scan_scores), so
        // the error word is read only on that rare path (its D2H was a blit launch + 4 us per call)
        MSV_HIP(hipStreamSynchronize(st));  // also: the pinned h_off is rewritten by the next call
        drain.armed = false;
        if (staged_scores) std::memcpy(scores, p->h_sc, n * sizeof(float));
        if (scan_scores(scores, n) == MSV_OK) return MSV_OK;
        const msv_status e = check_word(p, st, kHostErrWord);  // reads, clears and reports this call's bits
        return e != MSV_OK ? e : scan_scores(scores, n);
    }
    MSV_HIP(hipMemcpyAsync(scores, p->d_scores, n * sizeof(float), hipMemcpyDeviceToHost, st));
    MSV_HIP(hipMemcpyAsync(h_err, p->d_words + kHostErrWord, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    MSV_HIP(hipStreamSynchronize(st));  // also: the pinned h_off is rewritten by the next call
    drain.armed = false;
    if (*h_err == 0) return MSV_OK;
    return check_word(p, st, kHostErrWord);  // reads, clears and reports this call's error bits
}

msv_status msv_score_batch_async(msv_profile* p, const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                                 float* scores, uint64_t* ticket) {
    if (!p || !ticket || (n && (!offsets || !scores))) return MSV_ERR_INVALID_ARGUMENT;
    *ticket = 0;
    uint64_t maxL = 0;
    for (uint64_t s = 0; s < n; ++s) {
        if (offsets[s + 1] < offsets[s]) return MSV_ERR_INVALID_ARGUMENT;
        maxL = std::max<uint64_t>(maxL, offsets[s + 1] - offsets[s]);
    }
    const uint64_t total = n ? offsets[n] - offsets[0] : 0;
    if (total && !residues) return MSV_ERR_INVALID_ARGUMENT;
    // one launch per call: split larger batches (or use msv_score_batch)
    if (total >= kChunkBytes || n >= (1ull << 32) - (1ull << 24)) return MSV_ERR_INVALID_ARGUMENT;
    auto& a = p->async[p->next_ticket % kAsyncSlots];
    if (a.pending) return MSV_ERR_INVALID_ARGUMENT;  // that slot's call has not been waited for
    msv_status s = msv_profile_reserve_length(p, maxL);
    if (s != MSV_OK) return s;
    DeviceGuard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    if (!p->copy_stream) MSV_HIP(hipStreamCreateWithFlags(&p->copy_stream, hipStreamNonBlocking));
    if (!p->offsets_stream) MSV_HIP(hipStreamCreateWithFlags(&p->offsets_stream, hipStreamNonBlocking));
    if (!a.copied) MSV_HIP(hipEventCreateWithFlags(&a.copied, hipEventDisableTiming));
    if (!a.off_copied) MSV_HIP(hipEventCreateWithFlags(&a.off_copied, hipEventDisableTiming));
    if (!a.done) MSV_HIP(hipEventCreateWithFlags(&a.done, hipEventDisableTiming));
    if (!a.h_err) MSV_HIP(hipHostMalloc(reinterpret_cast<void**>(&a.h_err), 64, hipHostMallocDefault));
    MSV_HIP(ensure(a.d_res, a.res_cap, std::max<uint64_t>(total, 1)));
    MSV_HIP(ensure(a.d_off, a.off_cap, n + 1));
    float* const direct = n ? mapped_host(scores) : nullptr;
    if (!direct) MSV_HIP(ensure(a.d_sc, a.sc_cap, std::max<uint64_t>(n, 1)));
    MSV_HIP(ensure(a.d_ord, a.ord_cap, std::max<uint64_t>(n, 1)));
    if (a.h_cap < n + 1) {
        if (a.h_off) (void)hipHostFree(a.h_off);
        a.h_off = nullptr;
        a.h_cap = 0;
        MSV_HIP(hipHostMalloc(reinterpret_cast<void**>(&a.h_off), (n + 1) * sizeof(uint64_t), hipHostMallocDefault));
        a.h_cap = n + 1;
    }
    const uint64_t base = n ? offsets[0] : 0;
    for (uint64_t i = 0; i <= n; ++i) a.h_off[i] = n ? offsets[i] - base : 0;
    const int slot = static_cast<int>(&a - p->async);
    uint32_t* d_err = p->d_words + kErrWord + 1 + slot;
    // Consecutive calls alternate over two compute streams, so a call's kernel fills the CUs that the
    // previous call's drain tail frees instead of starting after the whole previous kernel.
    const bool odd = (p->next_ticket & 1) != 0;
    if (odd && !p->stream2) MSV_HIP(hipStreamCreateWithFlags(&p->stream2, hipStreamNonBlocking));
    hipStream_t cp = p->copy_stream, co = p->offsets_stream, cs = odd ? p->stream2 : p->stream;
    // On an error return after the first enqueue, copies reading this slot's pinned offsets (rewritten by
    // the slot's next call) may still be queued: drain the call's streams first.
    struct Drain {
        hipStream_t s[3];
        bool armed = true;
        ~Drain() {
            if (armed)
                for (hipStream_t x : s) (void)hipStreamSynchronize(x);
        }
    } drain{{co, cp, cs}};
    // copy streams: this call's inputs (they overlap the earlier calls' kernels on the compute streams).
    // Nothing but copies goes on them: a kernel there (the order, as in round 2) waits for the running MSV
    // grid to drain before it can start, and every later call's copies queued behind it.  The offsets
    // have a stream of their own, so the copy stream carries the residues back to back (cfg2: 83 us
    // each, which set the call rate with the offsets' 8 us copy and the gaps between them in the same
    // stream -- profiles/r03_cfg2_streamed_timeline.txt) and the order starts once the offsets land.
    MSV_HIP(hipMemcpyAsync(a.d_off, a.h_off, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, co));
    MSV_HIP(hipEventRecord(a.off_copied, co));
    if (total) MSV_HIP(hipMemcpyAsync(a.d_res, residues + base, total, hipMemcpyHostToDevice, cp));
    MSV_HIP(hipEventRecord(a.copied, cp));
    // compute stream: order, kernel, scores and the slot's error word back to the host (the order runs
    // in the previous call's drain tail: that call's kernel is on the other compute stream)
    MSV_HIP(hipStreamWaitEvent(cs, a.off_copied, 0));
    const bool sort = n && !order_needless(p, n, false);
    if (sort) {
        s = msv_order_longest_first(p, a.d_off, n, a.d_ord, cs);
        if (s != MSV_OK) return s;
    }
    MSV_HIP(hipStreamWaitEvent(cs, a.copied, 0));
    if (n) {
        s = launch_batch(p, total ? a.d_res : p->d_dummy, std::max<uint64_t>(total, 1), a.d_off, n,
                         sort ? a.d_ord : nullptr, direct ? direct : a.d_sc, cs, true, d_err);
        if (s != MSV_OK) return s;
        if (!direct) MSV_HIP(hipMemcpyAsync(scores, a.d_sc, n * sizeof(float), hipMemcpyDeviceToHost, cs));
    }
    if (!direct) {  // (direct: errors are read from the scores; nothing else follows the kernel)
        MSV_HIP(hipMemcpyAsync(a.h_err, d_err, sizeof(uint32_t), hipMemcpyDeviceToHost, cs));
        MSV_HIP(hipMemsetAsync(d_err, 0, sizeof(uint32_t), cs));
    }
    MSV_HIP(hipEventRecord(a.done, cs));
    drain.armed = false;
    a.direct = direct ? scores : nullptr;
    a.n = n;
    a.ticket = p->next_ticket++;
    a.pending = true;
    *ticket = a.ticket;
    return MSV_OK;
}

msv_status msv_profile_wait(msv_profile* p, uint64_t ticket) {
    if (!p || ticket == 0) return MSV_ERR_INVALID_ARGUMENT;
    for (auto& a : p->async) {
        if (!a.pending || a.ticket != ticket) continue;
        DeviceGuard g(p->device);
        if (!g.ok) return MSV_ERR_NO_DEVICE;
        MSV_HIP(hipEventSynchronize(a.done));
        a.pending = false;
        if (a.direct) {
            if (scan_scores(a.direct, a.n) == MSV_OK) return MSV_OK;
            // rare: classify from the bits the kernel latched in the slot's error word, and clear them
            const int slot = static_cast<int>(&a - p->async);
            uint32_t err = 0;
            MSV_HIP(hipMemcpyAsync(&err, p->d_words + kErrWord + 1 + slot, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   p->stream));
            MSV_HIP(hipMemsetAsync(p->d_words + kErrWord + 1 + slot, 0, sizeof(uint32_t), p->stream));
            MSV_HIP(hipStreamSynchronize(p->stream));
            const msv_status e = err_status(err);
            return e != MSV_OK ? e : scan_scores(a.direct, a.n);
        }
        return err_status(*a.h_err);
    }
    return MSV_ERR_INVALID_ARGUMENT;  // unknown ticket, or already waited for
}

// A grid of few sequences (one 64-lane wave each, at most this many waves over all profiles) runs as ONE
// launch: every profile's batch takes the latency layout of the grid's largest model, so each
// profile's launch lasts about as long as it would alone, and all of them run at once instead of
// queueing on the process's hardware queues (4 by default: 24 profiles x 3 sequences of 3,500
// residues, benchmark_MSV's shape, took 4.05 ms as 24 launches).
constexpr uint64_t kFusedMaxSeqs = 2048;

// The plan of `p` whose table is in variant v's layout (installing it as p->fused if none is).
static msv_status plan_in_layout(msv_profile* p, const msvk::Variant* v, const Plan** out) {
    for (const Plan* q : {&p->main, &p->lat, &p->mid, &p->fused})
        if (q->v == v) {
            *out = q;
            return MSV_OK;
        }
    const msv_status s = install_plan(p, v, p->fused);
    if (s != MSV_OK) return s;
    *out = &p->fused;
    return MSV_OK;
}

// The plan of `p` whose table is in cooperative variant cv's layout (installing it as p->coop_fused).
static msv_status coop_plan_in_layout(msv_profile* p, const msvk::CoopVariant* cv, const Plan** out) {
    for (const Plan* q : {&p->coop, &p->coop_fused})
        if (q->cv == cv) {
            *out = q;
            return MSV_OK;
        }
    const msv_status s = install_coop_table(p, cv, p->coop_fused);
    if (s != MSV_OK) return s;
    *out = &p->coop_fused;
    return MSV_OK;
}

// The cooperative variant a grid of n sequences x these profiles runs fused (grid_coop_fused), or nullptr:
// a grid of few sequences (n x profiles <= kFusedMaxSeqs), every profile with tr_E_C == tr_E_J and no
// forced variant, a variant covering the largest model -- and at most as many workgroups per launch (n x
// the launch's profiles) as the smallest coop_max_n of the listed profiles: the limit of the per-profile
// cooperative plan (about one workgroup fits a CU, so a launch of more is several rounds of the grid, and
// past ~2 rounds the cooperative plan loses).  coop_max_n = 0 (no cooperative plan, or
// msv_debug_set_coop_max_n(0)) turns the fused form off.  Residues read in place over PCIe
// (host_residues) keep the latency layout, as select_plan does.
static const msvk::CoopVariant* fused_coop_variant(msv_profile* const* profiles, uint32_t n_profiles, uint64_t n,
                                                   bool host_residues = false) {
    if (host_residues || n_profiles < 2 || n * n_profiles > kFusedMaxSeqs) return nullptr;
    uint32_t states = 0;
    uint64_t cap = ~0ull;
    for (uint32_t i = 0; i < n_profiles; ++i) {
        const msv_profile* p = profiles[i];
        if (p->force || std::memcmp(&p->tr_E_C, &p->tr_E_J, sizeof(float)) != 0) return nullptr;
        states = std::max(states, p->model_length - 1);
        cap = std::min(cap, p->coop_max_n);
    }
    if (static_cast<uint64_t>(std::min<uint32_t>(n_profiles, msvk::kGridMaxProfiles)) * n > cap) return nullptr;
    const msvk::CoopVariant* cv = pick_coop_variant(states);
    return cv && cv->grid_fn ? cv : nullptr;
}

// A grid of few sequences on the cooperative plan: ONE msv_coop_grid_kernel launch per 32 profiles, every
// profile's table in the cooperative layout of the grid's largest model, one workgroup per (profile,
// sequence).  The whole grid then lasts about as long as one sequence on one profile: benchmark_MSV's
// 24 profiles x 3 sequences of 3,500 residues run as 72 workgroups at once.  No dequeue counters.
static msv_status grid_coop_fused(msv_profile* const* profiles, uint32_t n_profiles, const msvk::CoopVariant* cv,
                                  const uint8_t* d_residues, uint64_t residues_len, const uint64_t* d_offsets,
                                  uint64_t n, const uint32_t* d_order, float* d_scores, hipStream_t cs) {
    if (residues_len >= (1ull << 32) || !d_offsets || (residues_len && !d_residues)) return MSV_ERR_INVALID_ARGUMENT;
    for (uint32_t first = 0; first < n_profiles; first += msvk::kGridMaxProfiles) {
        const uint32_t count = std::min(n_profiles - first, msvk::kGridMaxProfiles);
        msvk::GridArgs ga{};
        ga.profiles = count;
        ga.per_profile = static_cast<uint32_t>(n);
        for (uint32_t j = 0; j < count; ++j) {
            msv_profile* p = profiles[first + j];
            const Plan* plan = nullptr;
            const msv_status s = coop_plan_in_layout(p, cv, &plan);
            if (s != MSV_OK) return s;
            msvk::KernelArgs& a = ga.p[j];
            a.etab = plan->d_etab;
            a.residues = residues_len ? d_residues : p->d_dummy;
            a.offsets = d_offsets;
            a.order = d_order;
            a.lentab = p->d_lentab;
            a.scores = d_scores + static_cast<uint64_t>(first + j) * n;
            a.n = n;
            a.lentab_n = p->lentab_n;
            a.tr_B_Mk = p->tr_B_Mk;
            a.tr_E_C = p->tr_E_C;
            a.tr_E_J = p->tr_E_J;
            a.counter = p->d_words;  // (unused by the cooperative kernel)
            a.errors = p->d_words + kErrWord;
            a.stamps = nullptr;
        }
        void* params[] = {&ga};
        MSV_HIP(hipLaunchKernel(cv->grid_fn, dim3(count * ga.per_profile), dim3(static_cast<uint32_t>(cv->waves * 64)),
                                params, 0, cs));
    }
    return MSV_OK;
}

static msv_status grid_fused(msv_profile* const* profiles, uint32_t n_profiles, const msvk::Variant* v,
                             const uint8_t* d_residues, uint64_t residues_len, const uint64_t* d_offsets, uint64_t n,
                             const uint32_t* d_order, float* d_scores, hipStream_t cs) {
    if (residues_len >= (1ull << 32) || !d_offsets || (residues_len && !d_residues)) return MSV_ERR_INVALID_ARGUMENT;
    const uint32_t groups_per_block = static_cast<uint32_t>(v->waves * (64 / v->G) * v->streams);
    for (uint32_t first = 0; first < n_profiles; first += msvk::kGridMaxProfiles) {
        const uint32_t count = std::min(n_profiles - first, msvk::kGridMaxProfiles);
        msvk::GridArgs ga{};
        ga.profiles = count;
        ga.per_profile = static_cast<uint32_t>((n + groups_per_block - 1) / groups_per_block);
        int slot[msvk::kGridMaxProfiles];
        for (uint32_t j = 0; j < count; ++j) {
            msv_profile* p = profiles[first + j];
            const Plan* plan = nullptr;
            msv_status s = plan_in_layout(p, v, &plan);
            if (s != MSV_OK) return s;
            msvk::KernelArgs& a = ga.p[j];
            a.etab = plan->d_etab;
            a.residues = residues_len ? d_residues : p->d_dummy;
            a.offsets = d_offsets;
            a.order = d_order;
            a.lentab = p->d_lentab;
            a.scores = d_scores + static_cast<uint64_t>(first + j) * n;
            a.n = n;
            a.lentab_n = p->lentab_n;
            a.tr_B_Mk = p->tr_B_Mk;
            a.tr_E_C = p->tr_E_C;
            a.tr_E_J = p->tr_E_J;
            a.stamps = nullptr;
            MSV_HIP(p->kernels.acquire(cs, &slot[j]));
            a.counter = p->d_words + 2 * slot[j];
            a.errors = p->d_words + kErrWord;
            if (p->kernels.dirty[slot[j]]) MSV_HIP(hipMemsetAsync(a.counter, 0, 2 * sizeof(uint32_t), cs));
            p->kernels.dirty[slot[j]] = true;
        }
        MSV_HIP(msvk::launch_grid_variant(*v, ga, cs));
        for (uint32_t j = 0; j < count; ++j) {
            msv_profile* p = profiles[first + j];
            p->kernels.dirty[slot[j]] = false;
            MSV_HIP(p->kernels.release(slot[j], cs, lazy_stream(p, cs)));
        }
    }
    return MSV_OK;
}

// host_residues: d_residues is the device alias of page-locked host memory (msv_score_grid's in-place
// read): no cooperative plan (fused or per profile) and the per-profile launches take the zero-copy twins.
static msv_status score_grid_device(msv_profile* const* profiles, uint32_t n_profiles, const uint8_t* d_residues,
                                    uint64_t residues_len, const uint64_t* d_offsets, uint64_t n,
                                    const uint32_t* d_order, float* d_scores, void* stream, bool host_residues) {
    if (!profiles || n_profiles == 0) return MSV_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < n_profiles; ++i)
        if (!profiles[i] || profiles[i]->device != profiles[0]->device) return MSV_ERR_INVALID_ARGUMENT;
    if (n == 0) return MSV_OK;
    if (!d_scores) return MSV_ERR_INVALID_ARGUMENT;
    DeviceGuard g(profiles[0]->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    hipStream_t cs = stream ? static_cast<hipStream_t>(stream) : profiles[0]->stream;
    if (n_profiles > 1 && n * n_profiles <= kFusedMaxSeqs) {
        uint32_t states = 0;
        bool forced = false;
        uint32_t most = 0;  // the most times one handle is listed (each entry takes one of its counter slots)
        for (uint32_t i = 0; i < n_profiles; ++i) {
            states = std::max(states, profiles[i]->model_length - 1);
            forced |= profiles[i]->force;  // msv_profile_set_variant: that variant for every batch
            uint32_t same = 0;
            for (uint32_t j = 0; j < n_profiles; ++j) same += profiles[j] == profiles[i];
            most = std::max(most, same);
        }
        const msvk::CoopVariant* cv = fused_coop_variant(profiles, n_profiles, n, host_residues);
        if (cv)
            return grid_coop_fused(profiles, n_profiles, cv, d_residues, residues_len, d_offsets, n, d_order, d_scores, cs);
        // A fused launch holds one counter slot per entry until it ends: a handle listed more often than
        // it has slots would share a {next, waves left} pair between two sub-grids of one launch.
        forced |= most > static_cast<uint32_t>(kLaunchSlots);
        const msvk::Variant* fv = forced ? nullptr : pick_latency_variant(states);
        if (fv && fv->grid_fn)
            return grid_fused(profiles, n_profiles, fv, d_residues, residues_len, d_offsets, n, d_order, d_scores, cs);
    }
    hipEvent_t fork = nullptr;
    MSV_HIP(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    struct EventGuard {
        hipEvent_t e;
        ~EventGuard() { (void)hipEventDestroy(e); }
    } fork_guard{fork};
    MSV_HIP(hipEventRecord(fork, cs));
    // Largest models first: their launches are the longest, and with more streams than hardware queues
    // (HIP's default is 4) the launches queued behind them are the short ones.
    std::vector<uint32_t> launch_order(n_profiles);
    for (uint32_t i = 0; i < n_profiles; ++i) launch_order[i] = i;
    std::stable_sort(launch_order.begin(), launch_order.end(), [&](uint32_t x, uint32_t y) {
        return profiles[x]->model_length > profiles[y]->model_length;
    });
    for (const uint32_t i : launch_order) {
        msv_profile* p = profiles[i];
        if (!p->done) MSV_HIP(hipEventCreateWithFlags(&p->done, hipEventDisableTiming));
        hipStream_t ps = p->stream == cs ? cs : p->stream;
        if (ps != cs) MSV_HIP(hipStreamWaitEvent(ps, fork, 0));
        const msv_status s = launch_batch(p, d_residues, residues_len, d_offsets, n, d_order,
                                          d_scores + static_cast<uint64_t>(i) * n, ps, true, nullptr, host_residues);
        if (s != MSV_OK) return s;
        if (ps != cs) {
            MSV_HIP(hipEventRecord(p->done, ps));
            MSV_HIP(hipStreamWaitEvent(cs, p->done, 0));
        }
    }
    return MSV_OK;
}

msv_status msv_score_grid_device(msv_profile* const* profiles, uint32_t n_profiles, const uint8_t* d_residues,
                                 uint64_t residues_len, const uint64_t* d_offsets, uint64_t n,
                                 const uint32_t* d_order, float* d_scores, void* stream) {
    return score_grid_device(profiles, n_profiles, d_residues, residues_len, d_offsets, n, d_order, d_scores, stream,
                             false);
}

msv_status msv_score_grid(msv_profile* const* profiles, uint32_t n_profiles, const uint8_t* residues,
                          const uint64_t* offsets, uint64_t n, float* scores, void* stream) {
    if (!profiles || n_profiles == 0 || (n && (!offsets || !scores))) return MSV_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < n_profiles; ++i)
        if (!profiles[i] || profiles[i]->device != profiles[0]->device) return MSV_ERR_INVALID_ARGUMENT;
    if (n == 0) return MSV_OK;
    uint64_t maxL = 0;
    for (uint64_t s = 0; s < n; ++s) {
        if (offsets[s + 1] < offsets[s]) return MSV_ERR_INVALID_ARGUMENT;
        maxL = std::max<uint64_t>(maxL, offsets[s + 1] - offsets[s]);
    }
    const uint64_t bytes = offsets[n] - offsets[0];
    if (bytes && !residues) return MSV_ERR_INVALID_ARGUMENT;
    if (bytes >= kChunkBytes || n >= (1ull << 32) - (1ull << 24)) {  // huge batch: per profile, chunked
        for (uint32_t i = 0; i < n_profiles; ++i) {
            const msv_status s = msv_score_batch(profiles[i], residues, offsets, n, scores + i * n, stream);
            if (s != MSV_OK) return s;
        }
        return MSV_OK;
    }
    for (uint32_t i = 0; i < n_profiles; ++i) {
        const msv_status s = msv_profile_reserve_length(profiles[i], maxL);
        if (s != MSV_OK) return s;
    }
    msv_profile* p0 = profiles[0];
    DeviceGuard g(p0->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : shared_stream(p0->device);
    if (!st) st = p0->stream;
    if (!stream)
        for (uint32_t i = 0; i < n_profiles; ++i) profiles[i]->shared = st;  // lazy slot events (lazy_stream)
    // The first profile's staging buffers (a host call is synchronous, like msv_score_batch's use of
    // them): per-call hipMalloc/hipFree of four buffers cost more than the kernels of a small grid.
    // Page-locked residues are read in place and a page-locked destination is written by the kernels,
    // as in msv_score_batch.
    const uint64_t total = static_cast<uint64_t>(n_profiles) * n;
    const uint8_t* const zbase = (bytes && p0->zero_copy) ? mapped_host(residues) : nullptr;
    const uint8_t* const zres = zbase ? zbase + offsets[0] : nullptr;
    float* const direct = mapped_host(scores);
    if (!zres) MSV_HIP(ensure(p0->d_res, p0->d_res_cap, std::max<uint64_t>(bytes, 1)));
    MSV_HIP(ensure(p0->d_off, p0->d_off_cap, n + 1));
    MSV_HIP(ensure(p0->d_order, p0->d_order_cap, n));
    if (!direct) MSV_HIP(ensure(p0->d_scores, p0->d_scores_cap, total));
    if (p0->h_off_cap < n + 8) {  // pinned: the offsets H2D is a true async DMA
        if (p0->h_off) (void)hipHostFree(p0->h_off);
        p0->h_off = nullptr;
        p0->h_off_cap = 0;
        MSV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p0->h_off), (n + 8) * sizeof(uint64_t), hipHostMallocDefault));
        p0->h_off_cap = n + 8;
    }
    struct Drain {  // an early error return leaves nothing queued that reads h_off or the staging buffers
        hipStream_t st;
        bool armed = true;
        ~Drain() {
            if (armed) (void)hipStreamSynchronize(st);
        }
    } drain{st};
    for (uint64_t k = 0; k <= n; ++k) p0->h_off[k] = offsets[k] - offsets[0];
    const uint8_t* d_res = zres ? zres : p0->d_res;
    if (bytes && !zres) MSV_HIP(hipMemcpyAsync(p0->d_res, residues + offsets[0], bytes, hipMemcpyHostToDevice, st));
    MSV_HIP(hipMemcpyAsync(p0->d_off, p0->h_off, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    // (a fused cooperative grid runs one workgroup per sequence: no dequeue order to sort; residues read
    // in place never take it)
    const bool sort = fused_coop_variant(profiles, n_profiles, n, zres != nullptr) == nullptr;
    msv_status s = sort ? msv_order_longest_first(p0, p0->d_off, n, p0->d_order, st) : MSV_OK;
    if (s != MSV_OK) return s;
    float* const dsc = direct ? direct : p0->d_scores;
    s = score_grid_device(profiles, n_profiles, bytes ? d_res : p0->d_dummy, std::max<uint64_t>(bytes, 1), p0->d_off,
                          n, sort ? p0->d_order : nullptr, dsc, st, zres != nullptr);
    if (s != MSV_OK) return s;
    if (!direct) MSV_HIP(hipMemcpyAsync(scores, p0->d_scores, total * sizeof(float), hipMemcpyDeviceToHost, st));
    drain.armed = false;
    MSV_HIP(hipStreamSynchronize(st));  // pageable host buffers above
    // This call's errors show in its scores (+inf: bad residue, NaN: too long), so the profiles' latched
    // error words are read back only when there is one (a 4-byte read-back per profile is a blit kernel
    // plus a synchronisation: 24 profiles cost 0.9 ms, more than the whole grid's kernels).
    if (scan_scores(scores, total) == MSV_OK) return MSV_OK;
    msv_status first = MSV_OK;  // read back and clear EVERY profile's latched bits, report the first
    for (uint32_t i = 0; i < n_profiles; ++i) {
        s = msv_profile_check(profiles[i], st);
        if (first == MSV_OK) first = s;
    }
    return first != MSV_OK ? first : scan_scores(scores, total);
}

// Host restatement of msvk::msv_pvalue_of (kept textually parallel; tests compare both).
static double host_pvalue(float score, uint64_t L, float mu, float lambda) {
    if (L == 0) return 1.0;  // empty sequence: score -inf, and L log(p1) would be 0 * -inf
    const float p1 = static_cast<float>(L) / static_cast<float>(L + 1);
    const float nullsc = static_cast<float>(static_cast<double>(L) * std::log(static_cast<double>(p1)) +
                                            std::log(1.0 - static_cast<double>(p1)));
    const float bits = (score - nullsc) / 0.69314718055994529f;
    const double y = static_cast<double>(lambda) * (static_cast<double>(bits) - static_cast<double>(mu));
    const double ey = -std::exp(-y);
    return std::fabs(ey) < 5e-9 ? -ey : 1.0 - std::exp(ey);
}

msv_status msv_pvalues(const float* scores, const uint64_t* offsets, uint64_t n, float mu, float lambda,
                       double* pvalues) {
    if (n && (!scores || !offsets || !pvalues)) return MSV_ERR_INVALID_ARGUMENT;
    for (uint64_t i = 0; i < n; ++i) {
        if (offsets[i + 1] < offsets[i]) return MSV_ERR_INVALID_ARGUMENT;
        pvalues[i] = host_pvalue(scores[i], offsets[i + 1] - offsets[i], mu, lambda);
    }
    return MSV_OK;
}

msv_status msv_pvalues_device(int device, const float* d_scores, const uint64_t* d_offsets, uint64_t n, float mu,
                              float lambda, double* d_pvalues, void* stream) {
    if (n == 0) return MSV_OK;
    if (!d_scores || !d_offsets || !d_pvalues) return MSV_ERR_INVALID_ARGUMENT;
    DeviceGuard g(device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    MSV_HIP(msvk::launch_pvalues(d_scores, d_offsets, n, mu, lambda, d_pvalues, static_cast<hipStream_t>(stream)));
    return MSV_OK;
}

msv_status msv_score_batch_multi(msv_profile* const* profiles, uint32_t n_profiles, const uint8_t* residues,
                                 const uint64_t* offsets, uint64_t n, float* scores) {
    if (!profiles || n_profiles == 0 || (n && (!offsets || !scores))) return MSV_ERR_INVALID_ARGUMENT;
    for (uint32_t k = 0; k < n_profiles; ++k)
        if (!profiles[k]) return MSV_ERR_INVALID_ARGUMENT;
    if (n == 0) return MSV_OK;
    std::vector<uint64_t> b(n_profiles + 1);
    msv_status s = msv_shard_bounds(offsets, n, n_profiles, b.data());
    if (s != MSV_OK) return s;
    // One host thread per DISTINCT profile handle: a handle listed more than once scores its shards
    // one after another on its thread (a profile's staging buffers and streams serve one host
    // thread at a time).
    std::vector<msv_status> st(n_profiles, MSV_OK);
    std::vector<std::thread> workers;
    for (uint32_t k = 0; k < n_profiles; ++k) {
        bool first_use = true;
        for (uint32_t j = 0; j < k; ++j) first_use = first_use && profiles[j] != profiles[k];
        if (!first_use) continue;
        workers.emplace_back([&, k] {
            for (uint32_t j = k; j < n_profiles && st[k] == MSV_OK; ++j) {
                if (profiles[j] != profiles[k] || b[j + 1] == b[j]) continue;
                // offsets stay absolute: msv_score_batch rebases every piece on its first offset
                st[k] = msv_score_batch(profiles[k], residues, offsets + b[j], b[j + 1] - b[j], scores + b[j], nullptr);
            }
        });
    }
    for (auto& w : workers) w.join();
    for (uint32_t k = 0; k < n_profiles; ++k)
        if (st[k] != MSV_OK) return st[k];
    return MSV_OK;
}

msv_status msv_score_fasta_device(msv_profile* p, const msv_fasta_device* fasta, float* scores) {
    if (!p || !fasta) return MSV_ERR_INVALID_ARGUMENT;
    if (msv_fasta_device_device(fasta) != p->device) return MSV_ERR_INVALID_ARGUMENT;  // another GPU's memory
    const uint64_t n = msv_fasta_device_count(fasta);
    if (n == 0) return MSV_OK;
    if (!scores) return MSV_ERR_INVALID_ARGUMENT;
    msv_status s = msv_profile_reserve_length(p, msv_fasta_device_max_length(fasta));
    if (s != MSV_OK) return s;
    DeviceGuard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    MSV_HIP(ensure(p->d_scores, p->d_scores_cap, n));
    MSV_HIP(ensure(p->d_order, p->d_order_cap, n));
    const uint64_t* d_off = msv_fasta_device_offsets(fasta);
    s = msv_order_longest_first(p, d_off, n, p->d_order, p->stream);
    if (s != MSV_OK) return s;
    s = msv_score_batch_device(p, msv_fasta_device_codes(fasta), std::max<uint64_t>(msv_fasta_device_residues(fasta), 1),
                               d_off, n, p->d_order, p->d_scores, p->stream);
    if (s != MSV_OK) return s;
    MSV_HIP(hipMemcpyAsync(scores, p->d_scores, n * sizeof(float), hipMemcpyDeviceToHost, p->stream));
    return msv_profile_check(p, p->stream);
}

}  // extern "C"
