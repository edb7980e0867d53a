// vit_device.cpp -- C-ABI of the Viterbi stage (msv.h) on the HIP runtime.
//
// The reference parses insert emissions, transitions and STATS LOCAL VITERBI (Profile_HMM.cpp:86-87,
// 107-120) and never scores with them.  A msv_vit_profile holds the kernel-layout tables of one compiled
// variant (vit_kernel.hip), its own per-length {tr_loop, tr_move} table (host logf, MSV_HMM.cpp:59-64)
// and self-resetting dequeue counters (one pair per launch slot, launch_ring.h, so one profile may be
// driven from several streams at once); a batch -- typically the MSV filter's survivors, selected on the
// device -- is one persistent launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <new>
#include <vector>

#include "launch_ring.h"
#include "msv.h"
#include "msv_kernel.h"
#include "vit_kernel.h"

namespace {

constexpr uint32_t kDefaultMaxLength = 131072;
constexpr float kNinf = -std::numeric_limits<float>::infinity();
// d_words: [2k, 2k+1] = launch slot k's dequeue counters {next index, leavers} (zero between launches),
// [kErrWord] = sticky error bits of device launches (msv_vit_profile_check), [kHostErrWord] = the error bits
// of the synchronous host calls, which report and clear only their own, [kSelWord] = msv_vit_filter_batch's
// survivors count.
constexpr int kLaunchSlots = 8;
constexpr int kErrWord = 2 * kLaunchSlots;
constexpr int kHostErrWord = kErrWord + 1;
constexpr int kSelWord = kHostErrWord + 1;
constexpr int kWords = kSelWord + 1;

struct Guard {
    int prev = -1;
    bool ok = false;
    explicit Guard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~Guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

msv_status hip_status(hipError_t e) {
    if (e == hipSuccess) return MSV_OK;
    if (e == hipErrorOutOfMemory) return MSV_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return MSV_ERR_NO_DEVICE;
    return MSV_ERR_HIP;
}

#define VIT_HIP(call)                                \
    do {                                             \
        hipError_t e_ = (call);                      \
        if (e_ != hipSuccess) return hip_status(e_); \
    } while (0)

msv_status err_status(uint32_t err) {
    if (err & msvk::kErrBadResidue) return MSV_ERR_BAD_RESIDUE;
    if (err & msvk::kErrTooLong) return MSV_ERR_SEQUENCE_TOO_LONG;
    if (err & msvk::kErrBadOrder) return MSV_ERR_INVALID_ARGUMENT;  // a survivors entry outside the batch
    if (err & msvk::kErrTeamHang) return MSV_ERR_HIP;
    return err ? MSV_ERR_INVALID_ARGUMENT : MSV_OK;
}

// The automatic choice covering `states`: among the variants marked `pick` (one per S and insert mode, by
// measurement), the fewest slots.  Informative insert scores need an isc variant.
const vitk::VitVariant* pick_variant(uint32_t states, bool isc) {
    int n = 0;
    const vitk::VitVariant* all = vitk::vit_variants(&n);
    const vitk::VitVariant* best = nullptr;
    for (int i = 0; i < n; ++i) {
        const vitk::VitVariant& v = all[i];
        if (!v.pick || v.isc != isc || static_cast<uint32_t>(v.states()) < states) continue;
        if (!best || v.states() < best->states()) best = &v;
    }
    return best;
}

}  // namespace

struct msv_vit_profile {
    int device = 0;
    uint32_t model_length = 0;  // LENG + 1
    bool isc = false;
    float tr_B_Mk = 0, tr_E_C = 0, tr_E_J = 0;
    std::vector<float> msc, isc_tab, tsc;  // host copies (re-laid when the variant changes)
    const vitk::VitVariant* v = nullptr;
    uint32_t blocks = 0;                // persistent grid of a full launch
    float2* d_etab = nullptr;           // [20][S/2][64]
    float2* d_itab = nullptr;           // [20][S/2][64] (isc)
    float2* d_ttab = nullptr;           // [7][S/2][64]
    float2* d_lentab = nullptr;
    uint32_t lentab_n = 0;
    uint32_t* d_words = nullptr;        // kWords, see kLaunchSlots
    msvrt::LaunchRing<kLaunchSlots> kernels;  // the launch slots' streams and events
    hipStream_t stream = nullptr;
    hipStream_t bound = nullptr;        // msv_vit_profile_bind_stream: a caller stream kept alive while bound
    // msv_vit_score_batch / msv_vit_filter_batch staging
    uint8_t* d_res = nullptr;
    size_t res_cap = 0;
    uint64_t* d_off = nullptr;
    size_t off_cap = 0;
    float* d_sc = nullptr;
    size_t sc_cap = 0;
    float* d_msc_out = nullptr;
    size_t msc_out_cap = 0;
    uint32_t* d_sel = nullptr;
    size_t sel_cap = 0;
    uint32_t* d_ord = nullptr;
    size_t ord_cap = 0;
    hipEvent_t time_start = nullptr, time_stop = nullptr;  // msv_vit_debug_time_next_launch
    uint64_t* d_stamps = nullptr;                          // msv_vit_debug_set_stamps (tools only)
};

namespace {

template <typename T>
hipError_t ensure(T*& p, size_t& cap, size_t need) {
    if (need <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t n = std::max<size_t>(need, 1);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), n * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
}

// Kernel layouts of the variant's tables (vit_kernel.h): slot q of (virtual) lane l is state k = l * S + q + 1;
// chunk c of a lane holds slots 2c, 2c + 1 as one float2, lanes contiguous (a team's 64 * team virtual lanes;
// an odd S leaves the last chunk's second slot unused).
msv_status install(msv_vit_profile* p, const vitk::VitVariant* v) {
    const int S = v->S, C2 = v->chunks(), L64 = vitk::kLanes * v->team;
    const uint32_t M = p->model_length, K = M - 1;
    const size_t row2 = static_cast<size_t>(C2) * L64;
    auto state = [&](int l, int q) -> uint32_t { return static_cast<uint32_t>(l * S + q + 1); };
    std::vector<float2> et(vitk::kRows * row2), it(p->isc ? vitk::kRows * row2 : 0), tt(vitk::kTransitions * row2);
    for (int r = 0; r < vitk::kRows; ++r)
        for (int c = 0; c < C2; ++c)
            for (int l = 0; l < L64; ++l) {
                float e2[2], i2[2];
                for (int h = 0; h < 2; ++h) {
                    const uint32_t k = 2 * c + h < S ? state(l, 2 * c + h) : K + 1;  // (unused slot)
                    e2[h] = k <= K ? p->msc[static_cast<size_t>(r) * M + k] : kNinf;
                    i2[h] = (p->isc && k < K) ? p->isc_tab[static_cast<size_t>(r) * M + k] : 0.0f;
                }
                et[(r * C2 + c) * L64 + l] = make_float2(e2[0], e2[1]);
                if (p->isc) it[(r * C2 + c) * L64 + l] = make_float2(i2[0], i2[1]);
            }
    // per-slot transition arrays (vitk::MM_IN .. DD_IN); file order m->m m->i m->d i->m i->i d->m d->d
    enum { MM, MI, MD, IM, II, DM, DD };
    auto slot_t = [&](int j, uint32_t k) -> float {
        if (k > K) return kNinf;  // padding slots
        const float* tin = p->tsc.data() + static_cast<size_t>(k - 1) * 7;  // node k-1 -> node k
        const float* tout = p->tsc.data() + static_cast<size_t>(k) * 7;     // node k -> I(k)
        switch (j) {
            case vitk::MM_IN: return k >= 2 ? tin[MM] : kNinf;
            case vitk::IM_IN: return k >= 2 ? tin[IM] : kNinf;
            case vitk::DM_IN: return k >= 2 ? tin[DM] : kNinf;
            case vitk::MI: return k < K ? tout[MI] : kNinf;
            case vitk::II: return k < K ? tout[II] : kNinf;
            case vitk::MD_IN: return k >= 2 ? tin[MD] : kNinf;
            case vitk::DD_IN: return k >= 2 ? tin[DD] : kNinf;
        }
        return kNinf;
    };
    for (int j = 0; j < vitk::kTransitions; ++j)
        for (int c = 0; c < C2; ++c)
            for (int l = 0; l < L64; ++l)
                tt[(j * C2 + c) * L64 + l] = make_float2(slot_t(j, state(l, 2 * c)),
                                                         slot_t(j, 2 * c + 1 < S ? state(l, 2 * c + 1) : K + 1));

    float2 *de = nullptr, *di = nullptr, *dt = nullptr;
    hipError_t e;
    if ((e = hipMalloc(reinterpret_cast<void**>(&de), et.size() * sizeof(float2))) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&dt), tt.size() * sizeof(float2))) != hipSuccess ||
        (p->isc && (e = hipMalloc(reinterpret_cast<void**>(&di), it.size() * sizeof(float2))) != hipSuccess) ||
        (e = hipMemcpy(de, et.data(), et.size() * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(dt, tt.data(), tt.size() * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess ||
        (p->isc && (e = hipMemcpy(di, it.data(), it.size() * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess)) {
        (void)hipFree(de);
        (void)hipFree(di);
        (void)hipFree(dt);
        return hip_status(e);
    }
    int per_cu = 0, cus = 0;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, v->fn, v->waves * 64, 0)) != hipSuccess ||
        (e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->device)) != hipSuccess) {
        (void)hipFree(de);
        (void)hipFree(di);
        (void)hipFree(dt);
        return hip_status(e);
    }
    // the previous tables may still be read by a launch in flight on any stream
    if (p->d_etab || p->d_ttab) (void)hipDeviceSynchronize();
    (void)hipFree(p->d_etab);
    (void)hipFree(p->d_itab);
    (void)hipFree(p->d_ttab);
    p->d_etab = de;
    p->d_itab = di;
    p->d_ttab = dt;
    p->v = v;
    p->blocks = static_cast<uint32_t>(std::max(1, per_cu) * std::max(1, cus));
    return MSV_OK;
}

hipStream_t stream_of(const msv_vit_profile* p, void* stream) {
    return stream ? static_cast<hipStream_t>(stream) : p->stream;
}

// Every launch takes the next counter slot (a slot whose previous launch ran on another stream is reused
// only after it: launch_ring.h), so launches of one profile on several streams never share a counter.
// `errors` is the word the kernel latches its error bits into (device launches: kErrWord; host calls:
// kHostErrWord).
msv_status launch(msv_vit_profile* p, const uint8_t* d_residues, const uint64_t* d_offsets, uint64_t n,
                  const uint32_t* d_select, const uint32_t* d_select_count, float* d_scores, hipStream_t st,
                  uint32_t* errors, hipEvent_t start = nullptr, hipEvent_t stop = nullptr) {
    if (n == 0) return MSV_OK;
    if (n >= (1ull << 32)) return MSV_ERR_INVALID_ARGUMENT;
    vitk::VitArgs a{};
    a.etab = p->d_etab;
    a.itab = p->d_itab ? p->d_itab : p->d_etab;
    a.ttab = p->d_ttab;
    a.residues = d_residues;
    a.offsets = d_offsets;
    a.select = d_select;
    a.select_count = d_select ? d_select_count : nullptr;
    a.lentab = p->d_lentab;
    a.scores = d_scores;
    a.errors = errors;
    a.n = n;
    a.lentab_n = p->lentab_n;
    a.tr_B_Mk = p->tr_B_Mk;
    a.tr_E_C = p->tr_E_C;
    a.tr_E_J = p->tr_E_J;
    a.stamps = p->d_stamps;
    // one wave (team) per sequence: no more workgroups than the items need (a device count is bounded by n)
    const uint64_t per_block = static_cast<uint64_t>(p->v->sequences_per_block());
    const uint64_t need = (n + per_block - 1) / per_block;
    const uint32_t blocks = static_cast<uint32_t>(std::min<uint64_t>(p->blocks, need));
    if (!start && !stop && (p->time_start || p->time_stop)) {
        start = p->time_start;
        stop = p->time_stop;
        p->time_start = p->time_stop = nullptr;
    }
    int k = 0;
    VIT_HIP(p->kernels.acquire(st, &k));
    a.counter = p->d_words + 2 * k;
    // a slot's counters are put back to zero by the last wave of every launch; a failed launch may leave
    // them dirty, so the slot's next launch resets them explicitly
    if (p->kernels.dirty[k]) VIT_HIP(hipMemsetAsync(a.counter, 0, 2 * sizeof(uint32_t), st));
    p->kernels.dirty[k] = true;
    VIT_HIP(vitk::vit_launch(*p->v, blocks, a, st, start, stop));
    p->kernels.dirty[k] = false;
    VIT_HIP(p->kernels.release(k, st, st == p->stream || (p->bound && st == p->bound)));
    return MSV_OK;
}

// Reads (and clears when set) one error word of the profile on `st`, synchronously.
msv_status read_errors(msv_vit_profile* p, int word, hipStream_t st) {
    uint32_t err = 0;
    VIT_HIP(hipMemcpyAsync(&err, p->d_words + word, sizeof(err), hipMemcpyDeviceToHost, st));
    VIT_HIP(hipStreamSynchronize(st));
    if (err) {
        VIT_HIP(hipMemsetAsync(p->d_words + word, 0, sizeof(uint32_t), st));
        VIT_HIP(hipStreamSynchronize(st));
    }
    return err_status(err);
}

}  // namespace

extern "C" {

void msv_vit_profile_destroy(msv_vit_profile* p) {
    if (!p) return;
    Guard g(p->device);
    (void)hipDeviceSynchronize();
    for (void* d : {static_cast<void*>(p->d_etab), static_cast<void*>(p->d_itab), static_cast<void*>(p->d_ttab),
                    static_cast<void*>(p->d_lentab), static_cast<void*>(p->d_words), static_cast<void*>(p->d_res),
                    static_cast<void*>(p->d_off), static_cast<void*>(p->d_sc), static_cast<void*>(p->d_msc_out),
                    static_cast<void*>(p->d_sel), static_cast<void*>(p->d_ord)})
        (void)hipFree(d);
    p->kernels.destroy();
    if (p->stream) (void)hipStreamDestroy(p->stream);
    delete p;
}

msv_status msv_vit_profile_reserve_length(msv_vit_profile* p, uint64_t max_length) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    if (max_length >= (1ull << 31)) return MSV_ERR_SEQUENCE_TOO_LONG;
    const uint32_t need = static_cast<uint32_t>(max_length) + 1;
    if (need <= p->lentab_n) return MSV_OK;
    Guard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    const uint32_t n = std::max(need, p->lentab_n * 2);
    std::vector<float2> host(n);
    for (uint32_t L = 0; L < n; ++L) msv_sequence_transitions(L, &host[L].x, &host[L].y);  // MSV_HMM.cpp:59-64
    float2* d = nullptr;
    VIT_HIP(hipMalloc(reinterpret_cast<void**>(&d), n * sizeof(float2)));
    hipError_t e = hipMemcpy(d, host.data(), n * sizeof(float2), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return hip_status(e);
    }
    if (p->d_lentab) {
        (void)hipDeviceSynchronize();
        (void)hipFree(p->d_lentab);
    }
    p->d_lentab = d;
    p->lentab_n = n;
    return MSV_OK;
}

msv_status msv_vit_profile_create(int device, const float* match_scores, const float* insert_scores,
                                  const float* transition_scores, uint32_t model_length, float tr_B_Mk, float tr_E_C,
                                  float tr_E_J, msv_vit_profile** out) {
    if (!match_scores || !transition_scores || !out || model_length < 2) return MSV_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    // The kernel leaves D(LENG) out of E, exact only while every transition it reads (nodes 1 .. LENG-1,
    // install) is <= 0 (then every D is bounded by an M of its row); log-probabilities always are.
    for (size_t k = 1; k + 1 < model_length; ++k)
        for (int t = 0; t < 7; ++t)
            if (!(transition_scores[k * 7 + t] <= 0.0f)) return MSV_ERR_INVALID_ARGUMENT;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return MSV_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return MSV_ERR_NO_DEVICE;
    const vitk::VitVariant* v = pick_variant(model_length - 1, insert_scores != nullptr);
    if (!v) return MSV_ERR_UNSUPPORTED_MODEL;
    Guard g(device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    auto* p = new (std::nothrow) msv_vit_profile;
    if (!p) return MSV_ERR_OUT_OF_MEMORY;
    p->device = device;
    p->model_length = model_length;
    p->isc = insert_scores != nullptr;
    p->tr_B_Mk = tr_B_Mk;
    p->tr_E_C = tr_E_C;
    p->tr_E_J = tr_E_J;
    const size_t M = model_length;
    p->msc.assign(match_scores, match_scores + 20 * M);
    if (insert_scores) p->isc_tab.assign(insert_scores, insert_scores + 20 * M);
    p->tsc.assign(transition_scores, transition_scores + 7 * M);
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = p->kernels.create_events()) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&p->d_words), kWords * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMemset(p->d_words, 0, kWords * sizeof(uint32_t))) != hipSuccess) {
        msv_vit_profile_destroy(p);
        return hip_status(e);
    }
    msv_status s = install(p, v);
    if (s == MSV_OK) s = msv_vit_profile_reserve_length(p, kDefaultMaxLength - 1);
    if (s != MSV_OK) {
        msv_vit_profile_destroy(p);
        return s;
    }
    *out = p;
    return MSV_OK;
}

msv_status msv_vit_profile_create_from_hmm(int device, const msv_hmm* hmm, int insert_mode, msv_vit_profile** out) {
    if (!hmm || !out) return MSV_ERR_INVALID_ARGUMENT;
    const size_t M = msv_hmm_model_length(hmm);
    std::vector<float> msc(20 * M), isc(20 * M), tsc(7 * M);
    float b, c, j;
    msv_status s = msv_hmm_viterbi_scores(hmm, insert_mode, msc.data(), isc.data(), tsc.data(), &b, &c, &j);
    if (s != MSV_OK) return s;
    return msv_vit_profile_create(device, msc.data(), insert_mode == MSV_INSERTS_LOG_ODDS ? isc.data() : nullptr,
                                  tsc.data(), static_cast<uint32_t>(M), b, c, j, out);
}

msv_status msv_vit_profile_describe(const msv_vit_profile* p, msv_vit_info* out) {
    if (!p || !out) return MSV_ERR_INVALID_ARGUMENT;
    std::memset(out, 0, sizeof(*out));
    out->model_length = p->model_length;
    out->states_per_lane = static_cast<uint32_t>(p->v->S);
    out->transitions_in_registers = static_cast<uint32_t>(p->v->ntreg);
    out->match_in_lds = p->v->elds ? 1u : 0u;
    out->insert_scores = p->v->isc ? 1u : 0u;
    out->waves_per_block = static_cast<uint32_t>(p->v->waves);
    out->waves_per_sequence = static_cast<uint32_t>(p->v->team);
    out->blocks = p->blocks;
    out->lds_bytes = static_cast<uint32_t>(p->v->lds_bytes);
    out->max_length = p->lentab_n ? p->lentab_n - 1 : 0;
    out->device = p->device;
    std::snprintf(out->variant, sizeof(out->variant), "%s", p->v->name);
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, p->v->fn) == hipSuccess) {
        out->scratch_bytes = static_cast<uint32_t>(fa.localSizeBytes);
        out->lds_bytes = static_cast<uint32_t>(fa.sharedSizeBytes);  // the kernel's own static LDS, exactly
    }
    return MSV_OK;
}

int msv_vit_variant_count(void) {
    int n = 0;
    vitk::vit_variants(&n);
    return n;
}

const char* msv_vit_variant_name(int i) {
    int n = 0;
    const vitk::VitVariant* all = vitk::vit_variants(&n);
    return (i >= 0 && i < n) ? all[i].name : "";
}

msv_status msv_vit_profile_set_variant(msv_vit_profile* p, const char* name) {
    if (!p || !name) return MSV_ERR_INVALID_ARGUMENT;
    int n = 0;
    const vitk::VitVariant* all = vitk::vit_variants(&n);
    for (int i = 0; i < n; ++i)
        if (std::strcmp(all[i].name, name) == 0) {
            if (all[i].isc != p->isc || static_cast<uint32_t>(all[i].states()) < p->model_length - 1)
                return MSV_ERR_UNSUPPORTED_MODEL;
            Guard g(p->device);
            if (!g.ok) return MSV_ERR_NO_DEVICE;
            return install(p, &all[i]);
        }
    return MSV_ERR_INVALID_ARGUMENT;
}

msv_status msv_vit_score_batch_device(msv_vit_profile* p, const uint8_t* d_residues, uint64_t residues_len,
                                      const uint64_t* d_offsets, uint64_t n, const uint32_t* d_select,
                                      const uint32_t* d_select_count, float* d_scores, void* stream) {
    if (!p || (n && (!d_offsets || !d_scores))) return MSV_ERR_INVALID_ARGUMENT;
    if (n && residues_len && !d_residues) return MSV_ERR_INVALID_ARGUMENT;
    if (d_select_count && !d_select) return MSV_ERR_INVALID_ARGUMENT;
    Guard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    return launch(p, d_residues, d_offsets, n, d_select, d_select_count, d_scores, stream_of(p, stream),
                  p->d_words + kErrWord);
}

msv_status msv_vit_profile_bind_stream(msv_vit_profile* p, void* stream) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (st == p->bound) return MSV_OK;
    Guard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    if (p->bound) VIT_HIP(p->kernels.flush(p->bound));  // the old stream loses its guarantee
    p->bound = st;
    return MSV_OK;
}

// Diagnostic (bench.py): the next launch updates these two HIP events with its own start and end
// (hipExtLaunchKernel), so a timed launch adds no marker packets to its stream.  Not in msv.h.
msv_status msv_vit_debug_time_next_launch(msv_vit_profile* p, void* start, void* stop) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    p->time_start = static_cast<hipEvent_t>(start);
    p->time_stop = static_cast<hipEvent_t>(stop);
    return MSV_OK;
}

// Diagnostic (tools/vit_timeline.py, not in msv.h): subsequent team-kernel launches write their timeline to
// d_stamps (4 uint64 per list entry, then 4 per wave; the caller sizes it), nullptr turns it off.
msv_status msv_vit_debug_set_stamps(msv_vit_profile* p, uint64_t* d_stamps) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    p->d_stamps = d_stamps;
    return MSV_OK;
}

msv_status msv_vit_profile_check(msv_vit_profile* p, void* stream) {
    if (!p) return MSV_ERR_INVALID_ARGUMENT;
    Guard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    return read_errors(p, kErrWord, stream_of(p, stream));
}

msv_status msv_vit_score_batch(msv_vit_profile* p, const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                               float* scores, void* stream) {
    if (!p || (n && (!offsets || !scores))) return MSV_ERR_INVALID_ARGUMENT;
    if (n == 0) return MSV_OK;
    const uint64_t base = offsets[0], total = offsets[n] - base;
    if (total && !residues) return MSV_ERR_INVALID_ARGUMENT;
    for (uint64_t s = 0; s < n; ++s)
        if (offsets[s + 1] < offsets[s]) return MSV_ERR_INVALID_ARGUMENT;
    uint64_t longest = 0;
    for (uint64_t s = 0; s < n; ++s) longest = std::max(longest, offsets[s + 1] - offsets[s]);
    Guard g(p->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    msv_status s = msv_vit_profile_reserve_length(p, longest);
    if (s != MSV_OK) return s;
    hipStream_t st = stream_of(p, stream);
    std::vector<uint64_t> off(offsets, offsets + n + 1);
    for (auto& o : off) o -= base;
    VIT_HIP(ensure(p->d_res, p->res_cap, total));
    VIT_HIP(ensure(p->d_off, p->off_cap, n + 1));
    VIT_HIP(ensure(p->d_sc, p->sc_cap, n));
    if (total) VIT_HIP(hipMemcpyAsync(p->d_res, residues + base, total, hipMemcpyHostToDevice, st));
    VIT_HIP(hipMemcpyAsync(p->d_off, off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    s = launch(p, p->d_res, p->d_off, n, nullptr, nullptr, p->d_sc, st, p->d_words + kHostErrWord);
    if (s != MSV_OK) return s;
    VIT_HIP(hipMemcpyAsync(scores, p->d_sc, n * sizeof(float), hipMemcpyDeviceToHost, st));
    return read_errors(p, kHostErrWord, st);
}

msv_status msv_filter_select_device(int device, const float* d_scores, const uint64_t* d_offsets,
                                    const uint32_t* d_order, uint64_t n, float mu, float lambda, double threshold,
                                    double* d_pvalues, uint32_t* d_selected, uint32_t* d_count, void* stream) {
    if (!d_count || (n && (!d_scores || !d_offsets || !d_selected))) return MSV_ERR_INVALID_ARGUMENT;
    if (n >= (1ull << 32)) return MSV_ERR_INVALID_ARGUMENT;
    // No default stream here: NULL would be the legacy null stream, unordered with the profiles' own
    // non-blocking streams that msv_score_batch_device / msv_vit_score_batch_device take for NULL.
    if (!stream) return MSV_ERR_INVALID_ARGUMENT;
    Guard g(device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    return hip_status(
        vitk::launch_select(d_scores, d_offsets, d_order, n, mu, lambda, threshold, d_pvalues, d_selected, d_count, st));
}

msv_status msv_vit_filter_batch(msv_profile* msv, msv_vit_profile* vit, const uint8_t* residues,
                                const uint64_t* offsets, uint64_t n, float msv_mu, float msv_lambda, double F1,
                                float* msv_scores, uint8_t* passed, float* vit_scores, uint64_t* n_passed) {
    if (!msv || !vit || (n && (!offsets || !msv_scores || !passed || !vit_scores)) || !n_passed)
        return MSV_ERR_INVALID_ARGUMENT;
    *n_passed = 0;
    if (n == 0) return MSV_OK;
    if (n >= (1ull << 32)) return MSV_ERR_INVALID_ARGUMENT;
    msv_kernel_info info{};
    msv_status s = msv_profile_describe(msv, &info);
    if (s != MSV_OK) return s;
    if (info.device != vit->device) return MSV_ERR_INVALID_ARGUMENT;
    const uint64_t base = offsets[0], total = offsets[n] - base;
    if (total && !residues) return MSV_ERR_INVALID_ARGUMENT;
    uint64_t longest = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (offsets[i + 1] < offsets[i]) return MSV_ERR_INVALID_ARGUMENT;
        longest = std::max(longest, offsets[i + 1] - offsets[i]);
    }
    if (total >= (1ull << 32) - (1ull << 20)) return MSV_ERR_INVALID_ARGUMENT;  // one launch per stage
    Guard g(vit->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    if ((s = msv_profile_reserve_length(msv, longest)) != MSV_OK) return s;
    if ((s = msv_vit_profile_reserve_length(vit, longest)) != MSV_OK) return s;
    hipStream_t st = vit->stream;
    std::vector<uint64_t> off(offsets, offsets + n + 1);
    for (auto& o : off) o -= base;
    VIT_HIP(ensure(vit->d_res, vit->res_cap, total));
    VIT_HIP(ensure(vit->d_off, vit->off_cap, n + 1));
    VIT_HIP(ensure(vit->d_sc, vit->sc_cap, n));
    VIT_HIP(ensure(vit->d_msc_out, vit->msc_out_cap, n));
    VIT_HIP(ensure(vit->d_sel, vit->sel_cap, n));
    VIT_HIP(ensure(vit->d_ord, vit->ord_cap, n));
    if (total) VIT_HIP(hipMemcpyAsync(vit->d_res, residues + base, total, hipMemcpyHostToDevice, st));
    VIT_HIP(hipMemcpyAsync(vit->d_off, off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    // MSV over every sequence, longest first
    if ((s = msv_order_longest_first(msv, vit->d_off, n, vit->d_ord, st)) != MSV_OK) return s;
    if ((s = msv_score_batch_device(msv, vit->d_res, total, vit->d_off, n, vit->d_ord, vit->d_msc_out, st)) != MSV_OK)
        return s;
    // survivors (P <= F1) -> Viterbi, all on the device; non-survivors keep -inf (0xff800000)
    VIT_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(vit->d_sc), static_cast<int>(0xff800000u), n, st));
    // survivors listed longest first (the MSV launch's order): the Viterbi launch's tail is its shortest ones
    if ((s = msv_filter_select_device(vit->device, vit->d_msc_out, vit->d_off, vit->d_ord, n, msv_mu, msv_lambda, F1,
                                      nullptr, vit->d_sel, vit->d_words + kSelWord, st)) != MSV_OK)
        return s;
    if ((s = launch(vit, vit->d_res, vit->d_off, n, vit->d_sel, vit->d_words + kSelWord, vit->d_sc, st,
                    vit->d_words + kHostErrWord)) != MSV_OK)
        return s;
    uint32_t count = 0;
    VIT_HIP(hipMemcpyAsync(msv_scores, vit->d_msc_out, n * sizeof(float), hipMemcpyDeviceToHost, st));
    VIT_HIP(hipMemcpyAsync(vit_scores, vit->d_sc, n * sizeof(float), hipMemcpyDeviceToHost, st));
    VIT_HIP(hipMemcpyAsync(&count, vit->d_words + kSelWord, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    std::vector<uint32_t> sel;
    VIT_HIP(hipStreamSynchronize(st));
    if (count) {
        sel.resize(count);
        VIT_HIP(hipMemcpyAsync(sel.data(), vit->d_sel, count * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        VIT_HIP(hipStreamSynchronize(st));
    }
    std::fill(passed, passed + n, static_cast<uint8_t>(0));
    for (uint32_t x : sel) passed[x] = 1;
    *n_passed = count;
    if ((s = msv_profile_check(msv, st)) != MSV_OK) return s;
    return read_errors(vit, kHostErrWord, st);
}

}  // extern "C"
