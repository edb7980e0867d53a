// vit_team.hip -- the Viterbi stage with one sequence per TEAM of W waves (round 5).
//
// Same recurrence and bits as vit_kernel.hip (msv.h; restated serially in oracle/msv_oracle.c
// oracle_vit_run_codes):
//     M(i,k) = max(M'(k-1)+tMM, I'(k-1)+tIM, D'(k-1)+tDM, B'+tBM) + msc[r][k]
//     I(i,k) = max(M'(k)+tMI, I'(k)+tII)                            (isc = 0: HMMER3's insert scores)
//     D(i,k) = max(M(k-1)+tMD, D(k-1)+tDD)                           <- within the row
//     E = max_k M(i,k);  J, C, N, B as MSV_HMM.cpp:100-112
//
// Why teams.  With one sequence per 64-lane wave, a lane holds S = LENG/64 states of M, I, D plus the
// seven per-state transition scores: 10 S registers.  At S = 22 (1400.hmm) two waves fit a SIMD and at
// S = 38 (2405.hmm) one, and a wave alone issues at most one VALU instruction per ~2.4 ns (half the SIMD's
// rate), so every stall of a row's serial tail (lazy-F, E ballot, J, B) is lost issue:
// profiles/r04_pmc_vit_cfg3_final.json (S = 22) 52% VALU busy, profiles/r05_pmc_vit_cfg5.json (S = 38)
// 39%.  A team spreads the row over W waves (virtual lane v = w * 64 + lane holds states v*S+1 .. v*S+S),
// so S drops by W and three waves share a SIMD (<= 168 VGPRs) -- waves of DIFFERENT teams, each hiding the
// others' stalls.
//
// Per row, the waves of a team exchange through LDS, with no workgroup barrier (a workgroup holds NT
// teams that never wait for each other):
//   * E record {E_w, stamp}: the wave's E max when some lane's E + tEJ beats J + loop, else -inf.  Every
//     wave reads all W and forms J = max(J + loop, max_w E_w + tEJ) -- the single-wave kernel's J bit for
//     bit (fl() is monotone, and a wave whose lanes all lose adds nothing) -- then N, B.
//   * boundary record {M, I, D, stamp} of wave w's last state (lane 63, slot S-1), for wave w+1: the
//     previous row's M/I/D of state k0-1 enter its first state's M through the same DPP shift as a lane
//     boundary (its lane 0 keeps the record's value as the shift's `old`), and the row's new M/D enter its
//     first D through lazy-F (below).  Wave w publishes it after its own D chain is final, so corrections
//     ripple left to right (one hop per wave; W = 2 has a single hop).
//   Each record is one 8- or 16-byte LDS store carrying its stamp (the team's row counter), polled by the
//   reader; row parity double-buffers the records (the all-to-all E exchange keeps the team within a row).
// Work that needs neither record is done between publishing and polling: the I update and the
// B-independent part of the next row's M, a_k = max(M'(k-1)+tMM, I'(k-1)+tIM) (2 adds + max, written in
// place over M'(k), which is dead by then; M(i,k) = max3(a_k, D'(k-1)+tDM, Bt) + msc then costs the same 6
// VALU as the single-wave max3 form).  So a hop is covered by ~6 VALU per state of the wave's own work.
//
// Lazy-F across waves: a wave's first D starts from -inf (lower bound) and is raised after the exchange
// with cand = max(M_left + tMD, D_left + tDD) in its lane 0, in the same pass that carries D across its
// own lane boundaries (vit_kernel.hip's early-exit lazy-F); the last wave does that pass after the
// exchange, wave 0 before publishing.  Bitwise: the lower bounds only ever rise to the serial chain's
// values.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "msv_kernel_impl.h"
#include "vit_kernel.h"

namespace vitk {

namespace {

constexpr float TNINF = -__builtin_inff();
constexpr int kTeamEarlyD = 8;  // slots of the unconditional first lazy-F pass (vit_kernel.hip kEarlyD)
constexpr int DPP_WSHR1 = 0x138;
// A poll that spins this long means the team's protocol broke (a bug, never data): the wave latches
// kErrTeamHang and leaves the kernel instead of holding the GPU (each poll is one LDS round trip, so this is
// well under a second).
constexpr uint32_t kSpinLimit = 1u << 23;

__device__ __forceinline__ float tshift(float last, float old) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(last), DPP_WSHR1, 0xF, 0xF, false));
}
__device__ __forceinline__ bool tany(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// One team's exchange area (row parity p = row counter & 1).
template <int W>
struct TeamX {
    float4 b[2][W];  // boundary records {M, I, D, stamp} of wave w's last state
    float2 e[2][W];  // E records {E_w, stamp}
    float2 next[2];  // the team's sequence k: {item, k} (bits) at parity k & 1
};

// LDS accesses of the exchange: volatile native vectors, so every poll is a fresh single ds_read and every
// record is ONE ds_write (its stamp rides with the data: a reader that sees the stamp sees the record).  This
// relies on one lane's aligned 16-byte (boundary) and 8-byte (E, next) LDS access being single-copy atomic; only
// lane 0's copy of a boundary is used (the DPP shift's `old` for wave 1's lane 0) and lane 0's stamp is the one
// compared.  tests/test_team_exchange_isa.py checks in the gfx950 ISA that each record is one ds_write_b128 /
// ds_write_b64 and each poll one ds_read_b128 / ds_read_b64 comparing that load's last dword.  (Stamping every
// 8-byte half instead, which needs only 64-bit atomicity, was built in seven forms and measured 3-9% slower on
// cfg5's survivors: profiles/r06_ab/README.md.)
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))
__device__ __forceinline__ v4f lds_read4(const float4* p) { return *(const volatile LDS_AS v4f*)(p); }
__device__ __forceinline__ v2f lds_read2(const float2* p) { return *(const volatile LDS_AS v2f*)(p); }
__device__ __forceinline__ void lds_write4(float4* p, v4f v) { *(volatile LDS_AS v4f*)(p) = v; }
__device__ __forceinline__ void lds_write2(float2* p, v2f v) { *(volatile LDS_AS v2f*)(p) = v; }
__device__ __forceinline__ uint32_t ufirst(float x) { return __builtin_amdgcn_readfirstlane(__float_as_uint(x)); }
__device__ __forceinline__ uint64_t u64first(uint64_t x) {
    return (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32))) << 32) |
           __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x));
}

}  // namespace

// W waves per sequence, S states per lane (any S >= 2), match scores staged in LDS (ELDS) or read from L2
// each row, NT teams per workgroup.  Transitions: all seven arrays in VGPRs, or (LA = 1) the four of
// phase A (MM_IN, IM_IN, MI, II) in LDS, read chunk by chunk in phase A -- 4 S fewer VGPRs, so that the
// two-wave teams fit three waves per SIMD; LA = 2 also DM_IN (phase B, read a chunk ahead).  DD_IN and
// MD_IN (the D chain and lazy-F) stay in VGPRs.
template <int W, int S, bool ELDS, int NT, int LA = 0>
__global__ __launch_bounds__(NT * W * 64) void vit_team_kernel(const VitArgs a) {
    static_assert(S >= 2 && W >= 1 && W <= 4, "team shape");  // W = 1: one wave per sequence, no exchange
    constexpr int C2 = (S + 1) / 2;  // float2 chunks per lane (an odd S leaves the last .y unused)
    constexpr int VL = W * kLanes;   // virtual lanes of a team
    constexpr int ROW2 = C2 * VL;    // float2 per table row
    // Rows two per loop trip (the one-row loop copies values at its back edge) for the teams with phase-A
    // transitions in LDS: cfg5's survivors -2.9% (profiles/r05_ab_vit_team_two_rows.jsonl); the W = 1 S = 22
    // pick and the all-VGPR teams spill with two rows' register assignments (20-29 VGPRs).
    constexpr bool TWO_ROWS = W > 1 && LA > 0;
    __shared__ float2 etab_s[ELDS ? kRows * ROW2 : 1];
    // phase A's pairs as float4 {MM, IM} and {MI, II} per chunk (one ds_read_b128 each), DM_IN as float2
    __shared__ float4 tpa_s[LA ? 2 * C2 * VL : 1];
    constexpr int C4 = (C2 + 1) / 2;  // DM_IN chunk pairs (LA = 2): chunks 2p, 2p + 1 as one float4
    __shared__ float4 tdm_s[LA == 2 ? C4 * VL : 1];
    __shared__ TeamX<W> tx_s[NT];
    const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();  // (a.stamps only)
    // the list's length, at most n: a device count beyond the batch is latched (kErrBadOrder) and clamped, so no
    // wave reads the list past its n entries
    uint64_t total = a.n;
    if (a.select_count) {
        const uint64_t c = *a.select_count;
        if (c > a.n && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.errors, msvk::kErrBadOrder);
        total = c < a.n ? c : a.n;
    }
    if (static_cast<uint64_t>(blockIdx.x) * NT >= total) {
        // no sequence for this workgroup (vit_kernel.hip: a device-count launch sized for n): leave at once,
        // counted as its NT * W waves
        if (threadIdx.x == 0 && atomicAdd(a.counter + 1, static_cast<uint32_t>(NT * W)) == (gridDim.x - 1) * NT * W) {
            atomicExch(a.counter, 0u);
            atomicExch(a.counter + 1, 0u);
        }
        return;
    }
    const int lane = threadIdx.x & 63;
    // (readfirstlane: the wave's index is wave-uniform, so branches on it are scalar)
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int team = wv / W, w = wv % W;
    const int vl = w * kLanes + lane;
    TeamX<W>& tx = tx_s[team];

    if constexpr (ELDS)
        for (int i = threadIdx.x; i < kRows * ROW2; i += NT * W * 64) etab_s[i] = a.etab[i];
    if constexpr (LA) {
        for (int i = threadIdx.x; i < 2 * C2 * VL; i += NT * W * 64) {
            const int pr = i / (C2 * VL), r = i % (C2 * VL);
            const float2 x = a.ttab[(pr ? MI : MM_IN) * C2 * VL + r], y = a.ttab[(pr ? II : IM_IN) * C2 * VL + r];
            tpa_s[i] = make_float4(x.x, x.y, y.x, y.y);
        }
        if constexpr (LA == 2)
            for (int i = threadIdx.x; i < C4 * VL; i += NT * W * 64) {
                const int pc = i / VL, l = i % VL;
                const float2 x = a.ttab[(DM_IN * C2 + 2 * pc) * VL + l];
                const float2 y = 2 * pc + 1 < C2 ? a.ttab[(DM_IN * C2 + 2 * pc + 1) * VL + l] : make_float2(0.f, 0.f);
                tdm_s[i] = make_float4(x.x, x.y, y.x, y.y);
            }
    }
    for (int i = threadIdx.x; i < static_cast<int>(NT * sizeof(TeamX<W>) / 4); i += NT * W * 64)
        reinterpret_cast<uint32_t*>(tx_s)[i] = 0xFFFFFFFFu;  // no stamp matches
    __syncthreads();
    const uint64_t t_staged = __builtin_amdgcn_s_memrealtime();

    float tr[kTransitions][S];
#pragma unroll
    for (int j = 0; j < kTransitions; ++j) {
        if (LA && (j == MM_IN || j == IM_IN || j == MI || j == II)) continue;
        if (LA == 2 && j == DM_IN) continue;
#pragma unroll
        for (int c = 0; c < C2; ++c) {
            const float2 t = a.ttab[(j * C2 + c) * VL + vl];
            tr[j][2 * c] = t.x;
            if (2 * c + 1 < S) tr[j][2 * c + 1] = t.y;
        }
    }
    // LA: an opaque zero renewed every row keeps the compiler from hoisting the loop-invariant LDS reads of
    // the phase-A arrays out of the row loop into VGPRs (which would undo them)
    uint32_t rz = 0;

    const uint32_t nteams = gridDim.x * NT;
    uint32_t item = blockIdx.x * NT + team;  // first sequence static
    uint32_t k = 0;                          // the team's sequence ordinal
    uint32_t rc = 0;                         // the team's row counter (record stamps)
    const bool sameEJ = __float_as_uint(a.tr_E_C) == __float_as_uint(a.tr_E_J);
    const bool leader = w == 0 && lane == 0;

    // E records of row stamp `st`: publish this wave's E_w (lane 0: one store), and read the other waves'
    // (polling their stamps), returning max_w E_w.
    auto publish_e = [&](float Ew, uint32_t st) {
        if constexpr (W > 1)
            if (lane == 0) lds_write2(&tx.e[st & 1][w], v2f{Ew, __uint_as_float(st)});
    };
    bool hung = false;
    auto wait_e = [&](float Ew, uint32_t st_) -> float {
        const uint32_t st = __builtin_amdgcn_readfirstlane(st_);  // (keeps the stamp compare scalar)
        float m = Ew;
#pragma unroll
        for (int o = 1; o < W; ++o) {
            const int ww = (w + o) % W;
            v2f r;
            uint32_t spins = 0;
            do {
                r = lds_read2(&tx.e[st & 1][ww]);
                if (++spins > kSpinLimit) hung = true;
            } while (ufirst(r.y) != st && !hung);
            m = fmaxf(m, r.x);
        }
        return m;
    };

    while (item < total) {
        uint32_t tnext = 0;
        // The team's next sequence.  Teams (W > 1) take it once this sequence's first row has run: at the
        // launch's start every team's atomic hits the one counter at once, and taken first it would sit ahead
        // of the residue loads the first row waits for (cfg5 -1.4%, profiles/r05_ab_vit_take_late.jsonl); a
        // single wave (W = 1) takes it first (late was +0.7% on cfg3).
        bool taken = false;
        auto take = [&]() {
            taken = true;
            if (leader) tnext = atomicAdd(a.counter, 1u);
        };
        if constexpr (W == 1) take();
        // (readfirstlane: the sequence, its bounds and so every branch on them are wave-uniform -- scalar
        // branches and a scalar row counter, not exec-masked regions)
        const uint32_t s = __builtin_amdgcn_readfirstlane(a.select ? a.select[item] : item);
        const uint64_t t_seq = __builtin_amdgcn_s_memrealtime();
        const uint64_t o0 = u64first(a.offsets[s < a.n ? s : 0]);
        const uint64_t L = s < a.n ? u64first(a.offsets[s + 1]) - o0 : 0;
        if (s >= a.n || L == 0 || L >= a.lentab_n) {
            if (!taken) take();
            if (leader) {
                if (s >= a.n) {
                    atomicOr(a.errors, msvk::kErrBadOrder);  // a survivors entry outside the batch: skipped
                } else if (L == 0) {
                    a.scores[s] = TNINF;  // C_0 = -inf (MSV_HMM.cpp:86,112)
                } else {
                    a.scores[s] = __uint_as_float(0x7fc00000u);
                    atomicOr(a.errors, msvk::kErrTooLong);
                }
                if constexpr (W > 1)
                    lds_write2(&tx.next[(k + 1) & 1], v2f{__uint_as_float(nteams + tnext), __uint_as_float(k + 1)});
            }
            if constexpr (W > 1) {
                // one E exchange keeps the team within a sequence of each other (the `next` record's parity)
                publish_e(TNINF, rc);
                (void)wait_e(TNINF, rc);
                ++rc;
                if (hung) goto fail;
            }
        } else {
            const float2 lm = a.lentab[L];
            const float loop = lm.x, move = lm.y;
            const float tEJ = a.tr_E_J, tBM = a.tr_B_Mk;
            float M[S], I[S], D[S];
#pragma unroll
            for (int q = 0; q < S; ++q) M[q] = I[q] = D[q] = TNINF;
            float J = TNINF, Cp = TNINF, N = 0.0f, B = move;
            float lastM = TNINF, lastI = TNINF;        // this wave's last M, I of the previous row (lane shifts)
            float xM = TNINF, xI = TNINF, xD = TNINF;  // the left wave's last M, I, D of the previous row
            float Ew = TNINF;                          // this wave's E record of the previous row
            uint32_t maxcode = 0;
            const uint8_t* res = a.residues + o0;
            uint32_t cur = static_cast<uint64_t>(lane) < L ? res[lane] : 0u;
            uint32_t nxt = static_cast<uint64_t>(64 + lane) < L ? res[64 + lane] : 0u;

            // lazy-F: raise each lane's first D by `cand` (its left neighbour's last D + tDD, and in lane 0 of
            // a wave w > 0 the left wave's term), then carry the chain until no lane's first D changes.
            auto lazy_f = [&](float cand) {
                auto rest = [&]() {
#pragma unroll
                    for (int q = 1; q < S; ++q) D[q] = fmaxf(D[q], D[q - 1] + tr[DD_IN][q]);
                };
                auto again = [&]() {
                    cand = tshift(D[S - 1], TNINF) + tr[DD_IN][0];
                    while (tany(cand > D[0])) {
                        D[0] = fmaxf(D[0], cand);
                        rest();
                        cand = tshift(D[S - 1], TNINF) + tr[DD_IN][0];
                    }
                };
                if constexpr (kTeamEarlyD > 0 && S > kTeamEarlyD) {
                    // the first pass over slots 0 .. kTeamEarlyD-1 unconditionally, the rest only if some lane
                    // would still change (vit_kernel.hip: a slot that changes nowhere ends the chain)
                    D[0] = fmaxf(D[0], cand);
#pragma unroll
                    for (int q = 1; q < kTeamEarlyD; ++q) D[q] = fmaxf(D[q], D[q - 1] + tr[DD_IN][q]);
                    if (tany(D[kTeamEarlyD - 1] + tr[DD_IN][kTeamEarlyD] > D[kTeamEarlyD])) {
#pragma unroll
                        for (int q = kTeamEarlyD; q < S; ++q) D[q] = fmaxf(D[q], D[q - 1] + tr[DD_IN][q]);
                        again();
                    }
                } else {
                    while (tany(cand > D[0])) {
                        D[0] = fmaxf(D[0], cand);
                        rest();
                        cand = tshift(D[S - 1], TNINF) + tr[DD_IN][0];
                    }
                }
            };

            // One row.  Rows run two per loop trip where the registers allow it: over two rows the values
            // return to their registers by themselves (a one-row loop copied some at its back edge).
            auto row = [&](uint64_t i) -> bool {
                const uint32_t ph = static_cast<uint32_t>(i) & 63u;
                if (ph == 0 && i != 0) {
                    cur = nxt;
                    nxt = (i + 64 + lane < L) ? res[i + 64 + lane] : 0u;
                }

                if constexpr (W > 1)
                    if (i == 1) take();
                uint32_t code = __builtin_amdgcn_readlane(cur, ph);
                maxcode = code > maxcode ? code : maxcode;
                code = code < 19u ? code : 19u;
                // this row's match scores: from L2, all requested before the row's independent work; from LDS
                // (ELDS with LA), streamed a chunk ahead in phase B (fewer live VGPRs)
                constexpr bool EV_STREAM = ELDS && LA;
                float2 ev[C2];
                const float2* er;
                if constexpr (ELDS) er = etab_s + rz + code * ROW2 + vl;
                else er = a.etab + code * ROW2 + vl;
                if constexpr (!EV_STREAM) {
#pragma unroll
                    for (int c = 0; c < C2; ++c) ev[c] = er[c * VL];
                }
                // ---- phase A (the previous row's own values only): I(i, .), and a_q = max(M'(q-1)+tMM,
                // I'(q-1)+tIM) in place of M'(q) (M'(q) is dead once I(i, q) and a_{q+1} are made)
                if constexpr (LA) {
                    // chunk by chunk, highest first; each chunk's four pairs read one chunk ahead
                    asm volatile("" : "+v"(rz));
                    const float4* tl = tpa_s + rz + vl;
                    auto ld = [&](int c, float2 (&t)[4]) {
                        const float4 p0 = tl[c * VL], p1 = tl[(C2 + c) * VL];
                        t[0] = make_float2(p0.x, p0.y);
                        t[1] = make_float2(p0.z, p0.w);
                        t[2] = make_float2(p1.x, p1.y);
                        t[3] = make_float2(p1.z, p1.w);
                    };
                    float2 tc[4], tn[4];
                    ld(C2 - 1, tc);
#pragma unroll
                    for (int c = C2 - 1; c >= 0; --c) {
                        if (c > 0) ld(c - 1, tn);
#pragma unroll
                        for (int h = 1; h >= 0; --h) {
                            const int q = 2 * c + h;
                            if (q >= S) continue;
                            const float tmm = h ? tc[0].y : tc[0].x, tim = h ? tc[1].y : tc[1].x;
                            const float tmi = h ? tc[2].y : tc[2].x, tii = h ? tc[3].y : tc[3].x;
                            const float inew = fmaxf(M[q] + tmi, I[q] + tii);
                            if (q >= 1) M[q] = fmaxf(M[q - 1] + tmm, I[q - 1] + tim);
                            I[q] = inew;
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        if (c > 0)
#pragma unroll
                            for (int j = 0; j < 4; ++j) tc[j] = tn[j];
                    }
                } else {
#pragma unroll
                    for (int q = S - 1; q >= 1; --q) {
                        const float inew = fmaxf(M[q] + tr[MI][q], I[q] + tr[II][q]);
                        M[q] = fmaxf(M[q - 1] + tr[MM_IN][q], I[q - 1] + tr[IM_IN][q]);
                        I[q] = inew;
                    }
                    I[0] = fmaxf(M[0] + tr[MI][0], I[0] + tr[II][0]);
                }
                // pin phase A here, ahead of the polls (left alone, the compiler sinks it past them to its uses
                // in phase B, and the hop is waited for with nothing to issue)
#pragma unroll
                for (int q = 0; q < S; ++q) asm volatile("" : "+v"(M[q]), "+v"(I[q]));
                // ---- exchange of row i-1 (stamp rc-1)
                if (i != 0) {
                    const uint32_t st = __builtin_amdgcn_readfirstlane(rc - 1);
                    if (w > 0) {
                        // the left wave's boundary (its D chain final), then this wave's lazy-F of row i-1:
                        // its own lane boundaries and, in lane 0, D(k0) = max(M_left + tMD, D_left + tDD)
                        v4f r;
                        uint32_t spins = 0;
                        do {
                            r = lds_read4(&tx.b[st & 1][w - 1]);
                            if (++spins > kSpinLimit) hung = true;  // (checked after the E wait below)
                        } while (ufirst(r.w) != st && !hung);
                        xM = r.x;
                        xI = r.y;
                        xD = r.z;
                        lazy_f(fmaxf(tshift(D[S - 1], xD) + tr[DD_IN][0], tshift(TNINF, xM) + tr[MD_IN][0]));
                        if (w < W - 1 && lane == 63)
                            lds_write4(&tx.b[st & 1][w], v4f{lastM, lastI, D[S - 1], __uint_as_float(st)});
                    }
                    // J(i-1) from every wave's E record (the ballot used the same J + loop), N, B
                    const float Jn = J + loop;
                    J = fmaxf(Jn, wait_e(Ew, st) + tEJ);
                    if (hung) return false;
                    N = N + loop;
                    B = fmaxf(N, J) + move;
                }
                const float Bt = B + tBM;
                // ---- phase B: row i.  Slot 0 reads the previous row's state k0-1 through the lane shift (lane
                // 0 of a wave w > 0 keeps the left wave's record as the shift's `old`)
                const float sM = tshift(lastM, xM), sI = tshift(lastI, xI), sD = tshift(D[S - 1], xD);
                float tmm0, tim0;  // slot 0's entry transitions (LA: from LDS)
                if constexpr (LA) {
                    const float4 p0 = tpa_s[rz + vl];
                    tmm0 = p0.x;
                    tim0 = p0.z;
                } else {
                    tmm0 = tr[MM_IN][0];
                    tim0 = tr[IM_IN][0];
                }
                // DM_IN (LA = 2: from LDS, four slots per ds_read_b128, one pair ahead of use)
                const float4* tdm_l = tdm_s + rz + vl;
                float4 dmc = LA == 2 ? tdm_l[((S - 1) / 4) * VL] : make_float4(0.f, 0.f, 0.f, 0.f);
                auto tdm = [&](int q, float4 p4) -> float {
                    if constexpr (LA == 2) {
                        const int r = q & 3;
                        return r == 0 ? p4.x : r == 1 ? p4.y : r == 2 ? p4.z : p4.w;
                    } else {
                        return tr[DM_IN][q];
                    }
                };
                // the lane's last M first, so it can cross to the next lane for that lane's first D
                if constexpr (EV_STREAM) ev[C2 - 1] = er[(C2 - 1) * VL];
                const float mlast = fmaxf(fmaxf(M[S - 1], D[S - 2] + tdm(S - 1, dmc)), Bt) +
                                    (((S - 1) & 1) ? ev[(S - 1) / 2].y : ev[(S - 1) / 2].x);
                if constexpr (EV_STREAM) ev[0] = er[0];
                float E = mlast;
                {
                    float pd = sD, mn = tshift(mlast, TNINF), dn = TNINF;
                    if constexpr (LA == 2) dmc = tdm_l[0];
                    float4 dmn = dmc;
#pragma unroll
                    for (int q = 0; q < S; ++q) {
                        if constexpr (LA == 2) {
                            if ((q & 3) == 0) {
                                if (q > 0) dmc = dmn;
                                if (q / 4 + 1 < C4) dmn = tdm_l[(q / 4 + 1) * VL];
                            }
                        }
                        if constexpr (EV_STREAM) {
                            if ((q & 1) == 0 && q / 2 + 1 < C2 - 1) ev[q / 2 + 1] = er[(q / 2 + 1) * VL];
                        }
                        if constexpr (LA == 2 || EV_STREAM) {
                            if ((q & 1) == 0) __builtin_amdgcn_sched_barrier(0);
                        }
                        const float od = D[q];
                        float m;
                        if (q == S - 1) {
                            m = mlast;
                        } else {
                            const float aq = q == 0 ? fmaxf(sM + tmm0, sI + tim0) : M[q];
                            m = fmaxf(fmaxf(aq, pd + tdm(q, dmc)), Bt) + ((q & 1) ? ev[q / 2].y : ev[q / 2].x);
                            E = fmaxf(E, m);
                        }
                        const float d = q ? fmaxf(mn + tr[MD_IN][q], dn + tr[DD_IN][q]) : mn + tr[MD_IN][0];
                        M[q] = m;
                        D[q] = d;
                        pd = od;
                        mn = m;
                        dn = d;
                    }
                }
                // ---- end of row i: the E record (every wave); wave 0's D chain is final after its own lazy-F,
                // so it publishes its boundary at once (the other waves after the next exchange)
                Ew = tany(E + tEJ > J + loop) ? msvk::group_max<64>(E) : TNINF;
                if (!sameEJ) Cp = fmaxf(Cp + loop, E + a.tr_E_C);
                publish_e(Ew, rc);
                lastM = M[S - 1];
                lastI = I[S - 1];
                if (w == 0) {
                    lazy_f(tshift(D[S - 1], TNINF) + tr[DD_IN][0]);
                    if (W > 1 && lane == 63)
                        lds_write4(&tx.b[rc & 1][0], v4f{lastM, lastI, D[S - 1], __uint_as_float(rc)});
                }
                ++rc;
                return true;
            };
            uint64_t i = 0;
            if constexpr (TWO_ROWS) {
                for (; i + 1 < L; i += 2)
                    if (!row(i) || !row(i + 1)) goto fail;
            }
            for (; i < L; ++i)
                if (!row(i)) goto fail;
            if (!taken) take();  // (W > 1: a one-row sequence)
            if (W > 1 && leader)  // the team's next sequence (its atomic returned long ago)
                lds_write2(&tx.next[(k + 1) & 1], v2f{__uint_as_float(nteams + tnext), __uint_as_float(k + 1)});
            // J(L-1); the score C(L) + tr_move, C == J when tr_E_C == tr_E_J (MSV_HMM.cpp:49-53,112)
            J = fmaxf(J + loop, wait_e(Ew, rc - 1) + tEJ);
            float sc;
            if (sameEJ) {
                sc = J + move;
            } else {
                const float cw = msvk::group_max<64>(Cp);
                publish_e(cw, rc);
                sc = wait_e(cw, rc) + move;
                ++rc;
            }
            if (hung) goto fail;
            if (leader) {
                if (maxcode >= 20u) {
                    a.scores[s] = __builtin_inff();
                    atomicOr(a.errors, msvk::kErrBadResidue);
                } else {
                    a.scores[s] = sc;
                }
                if (a.stamps) {  // diagnostic timeline (nullptr in production)
                    uint32_t hwid = 0;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
                    uint64_t* st = a.stamps + 4 * static_cast<uint64_t>(item);
                    st[0] = t_seq;
                    st[1] = __builtin_amdgcn_s_memrealtime();
                    st[2] = (static_cast<uint64_t>(hwid) << 32) | (blockIdx.x * NT * W + wv);
                    st[3] = L;
                }
            }
        }
        if constexpr (W == 1) {
            item = nteams + __builtin_amdgcn_readfirstlane(tnext);  // (lane 0's atomic)
        } else {
            v2f r;
            uint32_t spins = 0;
            do {
                r = lds_read2(&tx.next[(k + 1) & 1]);
                if (++spins > kSpinLimit) goto fail;
            } while (ufirst(r.y) != k + 1);
            item = ufirst(r.x);
            ++k;
        }
    }
    if (false) {
    fail:
        if (lane == 0) atomicOr(a.errors, msvk::kErrTeamHang);
    }
    if (a.stamps && lane == 0) {  // diagnostic: this wave's entry, tables staged, exit, XCC id
        uint32_t xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        uint64_t* st = a.stamps + 4 * (total + blockIdx.x * NT * W + wv);
        st[0] = t_entry;
        st[1] = t_staged;
        st[2] = __builtin_amdgcn_s_memrealtime();
        st[3] = xcc;
    }
    // the last wave to finish resets the slot's counters for its next launch
    if (lane == 0) {
        __threadfence();
        if (atomicAdd(a.counter + 1, 1u) == gridDim.x * NT * W - 1) {
            atomicExch(a.counter, 0u);
            atomicExch(a.counter + 1, 0u);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Team variants (vit_kernel.h VitVariant::team = W): appended to vit_variants() by vit_kernel.hip.
// ------------------------------------------------------------------------------------------------
#define VIT_TEAM_LA(W_, S_, ELDS_, NT_, LA_, PICK_, NAME_)                                              \
    VitVariant{S_,                                                                                     \
               kTransitions - ((LA_) == 2 ? 5 : (LA_) == 1 ? 4 : 0),                                   \
               ELDS_,                                                                                  \
               false,                                                                                  \
               (NT_) * (W_),                                                                           \
               PICK_,                                                                                  \
               reinterpret_cast<const void*>(&vit_team_kernel<W_, S_, ELDS_, NT_, LA_>),               \
               NAME_,                                                                                  \
               (ELDS_ ? kRows * ((S_) + 1) / 2 * (W_) * kLanes * 8 : 0) +                              \
                   ((LA_) ? 4 * (((S_) + 1) / 2) * (W_) * kLanes * 8 : 0) +                              \
                   ((LA_) == 2 ? (((S_) + 1) / 2 + 1) / 2 * (W_) * kLanes * 16 : 0) +                         \
                   (NT_) * static_cast<int>(sizeof(TeamX<W_>)),                                        \
               W_}
#define VIT_TEAM(W_, S_, ELDS_, NT_, PICK_, NAME_) VIT_TEAM_LA(W_, S_, ELDS_, NT_, 0, PICK_, NAME_)

// Round 6 keeps the band picks (`true`) and two W = 2 forms with every transition in VGPRs (the timeline test's
// and tools/vit_concurrent.py's tail companion); the other ~35 round-5 A/B forms (W = 3 / 4, match scores in
// LDS, one-row loops, the W = 1 S = 12..20 rows) are in git history with their timings in
// profiles/r05_team_tune_*.jsonl.
const VitVariant* vit_team_variants(int* count) {
    static const VitVariant all[] = {
        // three waves per SIMD (<= 168 VGPRs): a 12-wave workgroup of 6 teams, and a one-team workgroup
        VIT_TEAM(2, 11, false, 6, false, "vit_w2_s11_g"),
        VIT_TEAM(2, 11, false, 1, false, "vit_w2_s11_g1"),
        // W = 1 (one wave per sequence, no exchange): the team kernel's row (phase A / B) with the phase-A
        // transitions in LDS, three waves per SIMD where vit_kernel.hip fits two -- the 1,281-1,408 pick
        VIT_TEAM_LA(1, 22, true, 12, 1, true, "vit_w1_s22_ea"),
        // phase-A transitions in LDS: four waves per SIMD (<= 128 VGPRs, 16-wave workgroups of 8 teams) for
        // S = 12, 13 (1509.hmm 1.90-1.94 vs 2.22-2.30 ms, 1600.hmm 2.11 vs 2.19 ms,
        // profiles/r05_team_tune_s12_two_rows.jsonl), three for S = 14, 15 ...
        VIT_TEAM_LA(2, 12, false, 8, 1, true, "vit_w2_s12_ga4"),
        VIT_TEAM_LA(2, 13, false, 8, 1, true, "vit_w2_s13_ga4"),
        VIT_TEAM_LA(2, 14, false, 6, 1, true, "vit_w2_s14_ga"),
        VIT_TEAM_LA(2, 15, false, 6, 1, true, "vit_w2_s15_ga"),
        // ... and DM_IN in LDS too (`gb`) for S = 17..19 (profiles/r05_team_tune_bands_la.jsonl: 1901.hmm 2.55 vs
        // 2.85 ms, 2138 / 2207.hmm -3.5 / -5%, cfg5's survivors 21.5 vs 22.6 ms)
        VIT_TEAM_LA(2, 17, false, 6, 2, true, "vit_w2_s17_gb"),
        VIT_TEAM_LA(2, 18, false, 6, 2, true, "vit_w2_s18_gb"),
        VIT_TEAM_LA(2, 19, false, 6, 2, true, "vit_w2_s19_gb"),
    };
    *count = static_cast<int>(sizeof(all) / sizeof(all[0]));
    return all;
}

}  // namespace vitk
