// vit_kernel.hip -- the Viterbi stage of SURVEY 8(f)-4 as ONE persistent gfx950 kernel per batch.
//
// The reference parses everything a Viterbi filter needs (insert_emissions and the 7 transitions per node,
// data_readers/Profile_HMM.cpp:107-120; STATS LOCAL VITERBI, :86-87) and never uses it; its README
// (README.md:2-3) names Viterbi as the point of the project.  This kernel scores HMMER3's generic local
// Viterbi (p7_GViterbi's recurrence, multihit local mode) over that parse, with the MSV path's specials
// (tr_B_Mk entry, E->C/J, per-length N/C/J loop/move, MSV_HMM.cpp:49-64), usually on the MSV filter's
// survivors.  Restated serially in oracle/msv_oracle.c (oracle_vit_run_codes, test-only); parity
// against it is bitwise.  Row i, residue r, k = 1..LENG:
//     M(i,k) = max(M'(k-1)+tMM, I'(k-1)+tIM, D'(k-1)+tDM, B'+tBM) + msc[r][k]
//     I(i,k) = max(M'(k)+tMI, I'(k)+tII) + isc[r][k]       (isc = 0: HMMER3's insert scores)
//     D(i,k) = max(M(k-1)+tMD, D(k-1)+tDD)                    <- within the row: a serial chain
//     E = max_k M(i,k);  J, C, N, B as MSV                    (D(LENG) <= E always: every t <= 0)
// Each term is ONE float add and max is exact, so any evaluation order of the maxes gives the same bits.
//
// Mapping (gfx950):
//   * one sequence per 64-lane wave (the stage sees the filter's few survivors, so a sequence gets a whole
//     wave); lane l holds the S consecutive states l*S+1 .. l*S+S of M, I, D in VGPRs;
//   * residues are wave-uniform: one byte per lane per 64-row block (a block ahead), v_readlane per row, so
//     the row's control, the table row address and the bad-code check are scalar;
//   * per row: the previous row's last M/I/D cross one lane boundary by DPP (row_bcast:15 + row_shr:1);
//     a descending pass updates M and I in place (slot q reads the old q-1), the new last M crosses, and
//     an ascending pass runs the lane's D chain in place;
//   * the D chain across lanes is resolved lazily (Farrar's lazy-F): the pass starts each lane's chain
//     from -inf, then while any lane's incoming D(k-1)+tDD beats its first D, the lanes re-run
//     D_q = max(D_q, D_{q-1}+tDD).  Lower bounds only ever rise to the exact value and fl() is
//     monotone, so the result is the serial chain bit for bit;
//   * J is kept exact and wave-uniform, the 64-lane max of E taken only on rows where some lane's E + tEJ
//     beats J + loop; C is a per-lane partial, its 64-lane max taken once per sequence;
//   * match scores staged in LDS ([20][S/2][64] float2: each ds_read_b64 of a wave is contiguous) and the
//     7 transition arrays in VGPRs, or (large models) transitions in LDS and match scores from L2;
//   * persistent grid, first sequence static, then one atomic per sequence; the counter resets itself.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>
#include <vector>

#include "msv_kernel_impl.h"
#include "vit_kernel.h"

namespace vitk {

namespace {

constexpr float NINF = -__builtin_inff();
constexpr int kEarlyD = 8;  // slots of the unconditional first lazy-F pass before its early-exit test
// rows of S < kEarlyD: states (over whole-lane hops) of the unconditional first lazy-F passes
constexpr int kEarlyHopStates = 8;

__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
__device__ __forceinline__ uint64_t u64first(uint64_t x) {
    return (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32))) << 32) |
           __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x));
}

// Lane l-1's value into lane l (64 lanes); lane 0 keeps `old`'s lane 0, which its caller keeps at -inf
// (the dummy column k = 0).  One DPP move across the whole wave (wave_shr:1, bound_ctrl off: the lane
// without a source keeps `old`) instead of the row_bcast:15 + row_shr:1 pair.
constexpr int DPP_WAVE_SHR1 = 0x138;
__device__ __forceinline__ float shift64(float last, float old) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(last), DPP_WAVE_SHR1, 0xF, 0xF, false));
}

}  // namespace

// One chunk (two slots) of the M/I pass: the LDS-resident transition pairs among MM, IM, DM, MI, II
// (NM of them), the match and the insert scores.  And of the D pass: the LDS-resident MD, DD pairs.
template <int NM>
struct ChunkMI {
    float2 t[NM ? NM : 1];
    float2 e, i;
};
template <int ND>
struct ChunkD {
    float2 t[ND ? ND : 1];
};

// PD > 0: a chunk's LDS/L2 data is requested PD chunks ahead and every chunk is its own scheduling region
// (bounds the live loads: left alone, the scheduler hoists a whole row of loads and spills).
// ASC: the row as ONE ascending pass (D chain interleaved with the M/I work) instead of a descending M/I pass
// followed by an ascending D pass.
template <int S, int NTREG, bool ELDS, bool ISC, int WAVES, int PD, bool ASC>
__global__ __launch_bounds__(WAVES * 64) void vit_kernel(const VitArgs a) {
    static_assert(S >= 2 && S % 2 == 0, "S must be even");
    // Rows two per loop trip where the registers allow it (the copies at a one-row loop's back edge); the
    // long rows of the L2 variants (S > 24) keep one row per trip: two rows' register assignments did not
    // fit 256 VGPRs there (S = 38: 83-124 spilled VGPRs).
    constexpr bool TWO_ROWS = S <= 24;
    constexpr int C2 = S / 2;
    constexpr int ROW2 = C2 * kLanes;                     // float2 per table row
    constexpr int kEarlyHops = S < kEarlyD ? kEarlyHopStates / S : 0;
    constexpr int NTL = kTransitions - NTREG;             // transition arrays in LDS
    constexpr int NM = NTREG >= MD_IN ? 0 : MD_IN - NTREG;  // ... of them used by the M/I pass
    constexpr int ND = NTL - NM;                          // ... by the D pass
    __shared__ float2 etab_s[ELDS ? kRows * ROW2 : 1];
    __shared__ float2 ttab_s[NTL ? NTL * ROW2 : 1];
    __shared__ uint32_t exited_s;  // waves of this workgroup that have left (the exit count below)
    const int lane = threadIdx.x & 63;
    // (readfirstlane: wave-uniform, so the sequence, its bounds and every branch on them are scalar)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // the list's length, at most n: a device count beyond the batch is latched (kErrBadOrder) and clamped, so no
    // wave reads the list past its n entries
    uint64_t total = a.n;
    if (a.select_count) {
        const uint64_t c = *a.select_count;
        if (c > a.n && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.errors, msvk::kErrBadOrder);
        total = c < a.n ? c : a.n;
    }
    if (static_cast<uint64_t>(blockIdx.x) * WAVES >= total) {
        // no sequence for this workgroup (a device-count launch is sized for n, the count may be far less:
        // cfg2's 260 survivors of 10,000): no first item, and none of the queue's (it starts at the grid's
        // wave count) -- leave without staging the tables, counted like any other workgroup
        if (threadIdx.x == 0 && atomicAdd(a.counter + 1, 1u) == gridDim.x - 1) {
            atomicExch(a.counter, 0u);
            atomicExch(a.counter + 1, 0u);
        }
        return;
    }

    if constexpr (ELDS)
        for (int i = threadIdx.x; i < kRows * ROW2; i += WAVES * 64) etab_s[i] = a.etab[i];
    if constexpr (NTL > 0)
        for (int i = threadIdx.x; i < NTL * ROW2; i += WAVES * 64) ttab_s[i] = a.ttab[NTREG * ROW2 + i];
    if (threadIdx.x == 0) exited_s = 0;
    __syncthreads();

    // transition arrays 0 .. NTREG-1 live in VGPRs for the whole launch, NTREG .. 6 in LDS (re-read every row)
    float tr[NTREG ? NTREG : 1][S];
    if constexpr (NTREG > 0) {
#pragma unroll
        for (int j = 0; j < NTREG; ++j)
#pragma unroll
            for (int c = 0; c < C2; ++c) {
                const float2 t = a.ttab[(j * C2 + c) * kLanes + lane];
                tr[j][2 * c] = t.x;
                tr[j][2 * c + 1] = t.y;
            }
    }
    // `rz` is an opaque zero renewed every row: without it the compiler hoists the loop-invariant LDS loads
    // of the transitions out of the row loop into VGPRs (and spills them), undoing the LDS arrays.
    uint32_t rz = 0;
    auto tlds = [&](int j, int c) -> float2 { return ttab_s[rz + ((j - NTREG) * C2 + c) * kLanes + lane]; };
    auto tdd = [&](int q) -> float {  // DD into slot q
        if constexpr (NTREG == kTransitions) {
            return tr[DD_IN][q];
        } else {
            const float2 t = tlds(DD_IN, q / 2);
            return (q & 1) ? t.y : t.x;
        }
    };

    const uint32_t nwaves = gridDim.x * WAVES;
    const bool few = total <= nwaves;  // wave-uniform: a latency-bound launch (no wave takes a second sequence)
    uint32_t item = blockIdx.x * WAVES + wave;
    while (item < total) {
        const uint32_t s = __builtin_amdgcn_readfirstlane(a.select ? a.select[item] : item);
        const uint64_t o0 = u64first(a.offsets[s < a.n ? s : 0]);
        const uint64_t L = s < a.n ? u64first(a.offsets[s + 1]) - o0 : 0;
        if (s >= a.n) {
            // a survivors entry outside the batch (a caller's list): reported, never dereferenced
            if (lane == 0) atomicOr(a.errors, msvk::kErrBadOrder);
        } else if (L == 0) {
            if (lane == 0) a.scores[s] = NINF;  // C_0 = -inf, as MSV_HMM.cpp:86,112
        } else if (L >= a.lentab_n) {
            if (lane == 0) {
                a.scores[s] = __uint_as_float(0x7fc00000u);
                atomicOr(a.errors, msvk::kErrTooLong);
            }
        } else {
            const float2 lm = a.lentab[L];
            const float loop = lm.x, move = lm.y;
            float M[S], I[S], D[S];
#pragma unroll
            for (int q = 0; q < S; ++q) M[q] = I[q] = D[q] = NINF;
            float J = NINF, Cp = NINF;  // J exact (wave-uniform), C as per-lane partials
            // tr_E_C == tr_E_J (the MSV specials: both logf(0.5)) makes C the same recurrence as J from the same
            // start, so C == J bit for bit and the partials are not kept
            const bool sameEJ = __float_as_uint(a.tr_E_C) == __float_as_uint(a.tr_E_J);
            float N = 0.0f, B = move;
            float sM = NINF, sI = NINF, sD = NINF, sMn = NINF, sDn = NINF;  // shift registers, lane 0 = -inf
            uint32_t maxcode = 0;
            const uint8_t* res = a.residues + o0;
            uint32_t cur = static_cast<uint64_t>(lane) < L ? res[lane] : 0u;
            uint32_t nxt = static_cast<uint64_t>(64 + lane) < L ? res[64 + lane] : 0u;
            // One row (residue i).  Rows run two per loop trip: a row writes its new M into registers other
            // than the old ones (the old M(k) is read after the new one is made), so a one-row loop copied
            // the whole row back at its back edge (22 v_mov per row at S = 22); over two rows the values
            // return to their registers by themselves.
            // (always_inline: the row must be inlined into both loops for its arrays to stay in registers -- left to
            // the inliner, the second copy of the loop put M / I / D of S >= 14 in scratch, 40x slower)
            auto row = [&](uint64_t i, auto hops_c) __attribute__((always_inline)) {  // hops_c: the short-row hops
                const uint32_t ph = static_cast<uint32_t>(i) & 63u;
                if (ph == 0 && i != 0) {
                    cur = nxt;
                    nxt = (i + 64 + lane < L) ? res[i + 64 + lane] : 0u;
                }
                uint32_t code = __builtin_amdgcn_readlane(cur, ph);
                maxcode = code > maxcode ? code : maxcode;
                code = code < 19u ? code : 19u;
                if constexpr (NTL > 0) asm volatile("" : "+v"(rz));
                const float Bt = B + a.tr_B_Mk;
                const float2* er;
                if constexpr (ELDS) er = etab_s + code * ROW2 + lane;  // (one address space per variant)
                else er = a.etab + code * ROW2 + lane;
                const float2* ir = a.itab + code * ROW2 + lane;
                auto load_mi = [&](int c) {
                    ChunkMI<NM> k;
#pragma unroll
                    for (int j = 0; j < NM; ++j) k.t[j] = tlds(NTREG + j, c);
                    k.e = er[c * kLanes];
                    if constexpr (ISC) k.i = ir[c * kLanes];
                    return k;
                };
                auto load_d = [&](int c) {
                    ChunkD<ND> k;
#pragma unroll
                    for (int j = 0; j < ND; ++j) k.t[j] = tlds(kTransitions - ND + j, c);
                    return k;
                };
                auto Tm = [&](const ChunkMI<NM>& k, int j, int q) -> float {  // j in MM_IN .. II
                    if (j < NTREG) return tr[j < NTREG ? j : 0][q];
                    const float2 t = k.t[j >= NTREG ? j - NTREG : 0];
                    return (q & 1) ? t.y : t.x;
                };
                auto Td = [&](const ChunkD<ND>& k, int j, int q) -> float {  // j = MD_IN or DD_IN
                    if (j < NTREG) return tr[j < NTREG ? j : 0][q];
                    const float2 t = k.t[j - (kTransitions - ND) >= 0 ? j - (kTransitions - ND) : 0];
                    return (q & 1) ? t.y : t.x;
                };

                // the previous row's last states, from the lane on the left (k - 1 across the boundary)
                sM = shift64(M[S - 1], sM);
                sI = shift64(I[S - 1], sI);
                sD = shift64(D[S - 1], sD);

                float E = NINF;
                if constexpr (ASC) {
                    // ONE ascending pass: slot q's I and M read the previous row at q and q-1 (old values carried
                    // in three registers) and its D the new M(q-1) and D(q-1), so the D chain runs interleaved
                    // with the independent M/I work.  The lane's last M is made first (peeled) so it can cross
                    // to the next lane for that lane's first D.
                    const ChunkMI<NM> kl = load_mi(C2 - 1);
                    const float mlast = fmaxf(fmaxf(M[S - 2] + Tm(kl, MM_IN, S - 1), I[S - 2] + Tm(kl, IM_IN, S - 1)),
                                              fmaxf(D[S - 2] + Tm(kl, DM_IN, S - 1), Bt)) +
                                        kl.e.y;
                    sMn = shift64(mlast, sMn);
                    ChunkMI<NM> km[C2];
                    ChunkD<ND> kd[C2];
                    if constexpr (PD > 0) {
#pragma unroll
                        for (int c = 0; c < C2 && c < PD; ++c) {
                            if (c < C2 - 1) km[c] = load_mi(c);
                            if constexpr (ND > 0) kd[c] = load_d(c);
                        }
                    }
                    float pm = sM, pi = sI, pd = sD, mn = sMn, dn = NINF;
#pragma unroll
                    for (int c = 0; c < C2; ++c) {
                        if constexpr (PD > 0) {
                            if (c + PD < C2) {
                                if (c + PD < C2 - 1) km[c + PD] = load_mi(c + PD);
                                if constexpr (ND > 0) kd[c + PD] = load_d(c + PD);
                            }
                        } else {
                            if (c < C2 - 1) km[c] = load_mi(c);
                            kd[c] = load_d(c);
                        }
                        const ChunkMI<NM>& k = c == C2 - 1 ? kl : km[c];
                        const ChunkD<ND>& kdd = kd[c];
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int q = 2 * c + h;
                            const float om = M[q], oi = I[q], od = D[q];
                            float iv = fmaxf(om + Tm(k, MI, q), oi + Tm(k, II, q));
                            if constexpr (ISC) iv = iv + (h ? k.i.y : k.i.x);
                            const float m = q == S - 1 ? mlast
                                                       : fmaxf(fmaxf(pm + Tm(k, MM_IN, q), pi + Tm(k, IM_IN, q)),
                                                               fmaxf(pd + Tm(k, DM_IN, q), Bt)) +
                                                             (h ? k.e.y : k.e.x);
                            const float d = q ? fmaxf(mn + Td(kdd, MD_IN, q), dn + Td(kdd, DD_IN, q))
                                              : mn + Td(kdd, MD_IN, 0);
                            M[q] = m;
                            I[q] = iv;
                            D[q] = d;
                            pm = om;
                            pi = oi;
                            pd = od;
                            mn = m;
                            dn = d;
                            E = fmaxf(E, m);
                        }
                        if constexpr (PD > 0) __builtin_amdgcn_sched_barrier(0);
                    }
                } else {
                    // M/I pass, highest slot first: I(k) reads M'(k), I'(k) and M(k) reads M'(k-1), I'(k-1),
                    // D'(k-1), so every register is updated in place (no copies at the loop's back edge)
                    ChunkMI<NM> km[C2];
                    if constexpr (PD > 0) {
    #pragma unroll
                        for (int c = C2 - 1; c >= 0 && c >= C2 - PD; --c) km[c] = load_mi(c);
                    }
    #pragma unroll
                    for (int c = C2 - 1; c >= 0; --c) {
                        if constexpr (PD > 0) {
                            if (c - PD >= 0) km[c - PD] = load_mi(c - PD);
                        } else {
                            km[c] = load_mi(c);
                        }
                        const ChunkMI<NM>& k = km[c];
    #pragma unroll
                        for (int h = 1; h >= 0; --h) {
                            const int q = 2 * c + h;
                            float iv = fmaxf(M[q] + Tm(k, MI, q), I[q] + Tm(k, II, q));
                            if constexpr (ISC) iv = iv + (h ? k.i.y : k.i.x);
                            const float pm = q ? M[q - 1] : sM, pi = q ? I[q - 1] : sI, pd = q ? D[q - 1] : sD;
                            const float m = fmaxf(fmaxf(pm + Tm(k, MM_IN, q), pi + Tm(k, IM_IN, q)),
                                                  fmaxf(pd + Tm(k, DM_IN, q), Bt)) +
                                            (h ? k.e.y : k.e.x);
                            M[q] = m;
                            I[q] = iv;
                            E = fmaxf(E, m);
                        }
                        if constexpr (PD > 0) __builtin_amdgcn_sched_barrier(0);
                    }
                    // this row's M(k-1) for each lane's first slot
                    sMn = shift64(M[S - 1], sMn);
                    // D pass, lowest slot first (the chain D(k) = max(M(k-1)+tMD, D(k-1)+tDD)), each lane's
                    // chain started from -inf; lazy-F below carries D across the lane boundaries
                    ChunkD<ND> kd[C2];
                    if constexpr (PD > 0 && ND > 0) {
    #pragma unroll
                        for (int c = 0; c < C2 && c < PD; ++c) kd[c] = load_d(c);
                    }
    #pragma unroll
                    for (int c = 0; c < C2; ++c) {
                        if constexpr (PD > 0 && ND > 0) {
                            if (c + PD < C2) kd[c + PD] = load_d(c + PD);
                        } else {
                            kd[c] = load_d(c);
                        }
                        const ChunkD<ND>& k = kd[c];
    #pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int q = 2 * c + h;
                            D[q] = q ? fmaxf(M[q - 1] + Td(k, MD_IN, q), D[q - 1] + Td(k, DD_IN, q))
                                     : sMn + Td(k, MD_IN, 0);
                        }
                        if constexpr (PD > 0 && ND > 0) __builtin_amdgcn_sched_barrier(0);
                    }
                }
                // lazy-F: carry D across lane boundaries until no lane's first state changes
                sDn = shift64(D[S - 1], sDn);
                float cand = sDn + tdd(0);
                auto lazy_f = [&]() {
                    do {
                        D[0] = fmaxf(D[0], cand);
#pragma unroll
                        for (int q = 1; q < S; ++q) D[q] = fmaxf(D[q], D[q - 1] + tdd(q));
                        sDn = shift64(D[S - 1], sDn);
                        cand = sDn + tdd(0);
                    } while (wave_any(cand > D[0]));
                };
                if constexpr (S > kEarlyD) {
                    // With 64 lanes some D path crosses a lane boundary on nearly every row (1.00 correction
                    // passes per row on 1400.hmm), and it dies out within a few states (the last state a pass
                    // changes: median 6, 74% <= 7; tools/lazy_f_stats.py).  So the first pass runs
                    // unconditionally over slots 0 .. kEarlyD-1, and the rest of the lane only if some lane
                    // would still change at slot kEarlyD: a slot that changes nowhere stops the chain (every
                    // later D was computed from the same values), and then no lane's last D changed either,
                    // so no second pass is needed.  Same max/add sequence per state as the serial chain.
                    D[0] = fmaxf(D[0], cand);
#pragma unroll
                    for (int q = 1; q < kEarlyD; ++q) D[q] = fmaxf(D[q], D[q - 1] + tdd(q));
                    if (wave_any(D[kEarlyD - 1] + tdd(kEarlyD) > D[kEarlyD])) {
#pragma unroll
                        for (int q = kEarlyD; q < S; ++q) D[q] = fmaxf(D[q], D[q - 1] + tdd(q));
                        sDn = shift64(D[S - 1], sDn);
                        cand = sDn + tdd(0);
                        if (wave_any(cand > D[0])) lazy_f();
                    }
                } else if constexpr (kEarlyHops > 1 && decltype(hops_c)::value) {
                    // short rows of a latency-bound launch (at most one sequence per wave): the same first kEarlyD
                    // states of the chain as above, here over kEarlyHops lanes -- whole-lane passes with their
                    // lane shifts run unconditionally (a D path crossing lanes costs a ballot and a branch per hop
                    // on the row's chain otherwise), then the ballot once.  cfg2's survivors -6.5%, 200.hmm x 300
                    // -13%; with several sequences per wave the extra passes cost issue slots the other waves
                    // would use (100.hmm x 20k +11% with hops), so those launches keep the ballot first -- at
                    // +2-3% for the second copy of the row loop (profiles/r05_ab_vit_short_row_hops.jsonl)
#pragma unroll
                    for (int h = 0; h < kEarlyHops; ++h) {
                        D[0] = fmaxf(D[0], cand);
#pragma unroll
                        for (int q = 1; q < S; ++q) D[q] = fmaxf(D[q], D[q - 1] + tdd(q));
                        sDn = shift64(D[S - 1], sDn);
                        cand = sDn + tdd(0);
                    }
                    if (wave_any(cand > D[0])) lazy_f();
                } else {
                    if (__builtin_expect(wave_any(cand > D[0]), 0)) lazy_f();
                }
                // specials (MSV_HMM.cpp:107-110).  J = max(J + loop, max_k E + tEJ) is kept exact and
                // wave-uniform: the 64-lane max of E is taken only on rows where some lane's E + tEJ beats
                // J + loop (a new best segment forming; fl() is monotone, so max_l fl(E_l + t) = fl(max_l E_l
                // + t)).  Per-lane J partials (the MSV kernel's form) needed the 64-lane max of J on every row
                // after the first hit, and the filter's survivors are the sequences with hits.
                const float Jn = J + loop;
                J = __builtin_expect(wave_any(E + a.tr_E_J > Jn), 0) ? fmaxf(Jn, msvk::group_max<64>(E) + a.tr_E_J)
                                                                       : Jn;
                if (!sameEJ) Cp = fmaxf(Cp + loop, E + a.tr_E_C);
                N = N + loop;
                B = fmaxf(N, J) + move;
            };
            uint64_t i = 0;
            auto rows = [&](auto hops_c) __attribute__((always_inline)) {
                if constexpr (TWO_ROWS) {
                    for (; i + 1 < L; i += 2) {
                        row(i, hops_c);
                        row(i + 1, hops_c);
                    }
                }
                for (; i < L; ++i) row(i, hops_c);
            };
            // the row loop compiled twice where the hops apply, chosen per sequence (a scalar branch outside
            // the loop: a per-row branch between the two lazy-F forms cost ~3% on both)
            if constexpr (kEarlyHops > 1) {
                if (few) rows(std::true_type{});
                else rows(std::false_type{});
            } else {
                rows(std::false_type{});
            }
            const float sc = (sameEJ ? J : msvk::group_max<64>(Cp)) + move;
            if (lane == 0) {
                if (maxcode >= 20u) {
                    a.scores[s] = __builtin_inff();
                    atomicOr(a.errors, msvk::kErrBadResidue);
                } else {
                    a.scores[s] = sc;
                }
            }
        }
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(a.counter, 1u);
        item = nwaves + __builtin_amdgcn_readfirstlane(t);
    }
    // the last workgroup to finish resets the counters for the next launch on this profile.  One grid-level
    // atomic per workgroup (by its last wave, counted in LDS), not per wave: a device-count launch of few
    // survivors runs thousands of waves that find no work, and their same-address exit atomics delayed the
    // launch's end (cfg2 in place, 8,192 waves for 260 survivors: 0.223 -> 0.206 ms,
    // profiles/r05_ab_wg_exit.jsonl; the MSV and team kernels were neutral / +1.3% and keep a count per wave)
    if (lane == 0) {
        __threadfence();
        if (atomicAdd(&exited_s, 1u) == WAVES - 1 && atomicAdd(a.counter + 1, 1u) == gridDim.x - 1) {
            atomicExch(a.counter, 0u);
            atomicExch(a.counter + 1, 0u);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// MSV filter survivors: the P-value of every score and a STABLE stream compaction of the sequences with
// P <= threshold, in the given dequeue order -- three launches: (1) P-values and each 256-entry block's
// survivor count, (2) one workgroup turns the counts into exclusive prefixes (and the total), (3) each block
// writes its survivors at their exact rank.  O(n) in all (round 5 summed every block's predecessors in (3),
// O(blocks^2)).  With the MSV launch's longest-first order the Viterbi launch then takes its survivors exactly
// longest first, so its drain tail is its shortest sequences (an unordered append -- one atomic per wave,
// stretches of 64 in arrival order -- left long survivors in the last round of the persistent grid:
// cfg3 1.40 vs 1.26 ms, cfg5 21.6 vs 20.0 ms with the team kernels, profiles/r05_select_order.jsonl).
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int kSelBlock = 256;

__device__ __forceinline__ bool select_pass(const float* scores, const uint64_t* offsets, const uint32_t* order,
                                            uint64_t n, float mu, float lambda, double threshold, double* pvalues,
                                            uint64_t pos, uint32_t* idx) {
    if (pos >= n) return false;
    const uint64_t i = order ? order[pos] : pos;  // (a permutation: every sequence is visited once)
    *idx = static_cast<uint32_t>(i);
    const double p = msvk::msv_pvalue_of(scores[i], offsets[i + 1] - offsets[i], mu, lambda);
    if (pvalues) pvalues[i] = p;
    return p <= threshold;
}

// Block sum of one uint32 per thread (4 waves).
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* lds4) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) lds4[wv] = v;
    __syncthreads();
    const uint32_t t = lds4[0] + lds4[1] + lds4[2] + lds4[3];
    __syncthreads();
    return t;
}
}  // namespace

__global__ __launch_bounds__(kSelBlock) void vit_select_count_kernel(const float* __restrict__ scores,
                                                                     const uint64_t* __restrict__ offsets,
                                                                     const uint32_t* __restrict__ order, uint64_t n,
                                                                     float mu, float lambda, double threshold,
                                                                     double* __restrict__ pvalues,
                                                                     uint32_t* __restrict__ block_counts) {
    __shared__ uint32_t lds4[4];
    uint32_t idx = 0;
    const uint64_t pos = static_cast<uint64_t>(blockIdx.x) * kSelBlock + threadIdx.x;
    const bool pass = select_pass(scores, offsets, order, n, mu, lambda, threshold, pvalues, pos, &idx);
    const uint32_t c = block_sum(pass ? 1u : 0u, lds4);
    if (threadIdx.x == 0) block_counts[blockIdx.x] = c;
}

// Exclusive prefix sums of the block counts in place, and the total into *count: one workgroup, each thread a
// contiguous run of the counts (blocks <= 2^24 for n < 2^32, so a run is <= 16,384 entries).
constexpr int kScanBlock = 1024;
__global__ __launch_bounds__(kScanBlock) void vit_select_scan_kernel(uint32_t* __restrict__ block_counts,
                                                                    uint32_t blocks, uint32_t* __restrict__ count) {
    __shared__ uint32_t part_s[kScanBlock];
    const uint32_t per = (blocks + kScanBlock - 1) / kScanBlock;
    const uint32_t b0 = threadIdx.x * per, b1 = b0 + per < blocks ? b0 + per : blocks;
    uint32_t sum = 0;
    for (uint32_t j = b0; j < b1; ++j) sum += block_counts[j];
    part_s[threadIdx.x] = sum;
    __syncthreads();
    // Hillis-Steele inclusive scan of the 1,024 run sums
    for (int d = 1; d < kScanBlock; d <<= 1) {
        const uint32_t v = threadIdx.x >= static_cast<uint32_t>(d) ? part_s[threadIdx.x - d] : 0u;
        __syncthreads();
        part_s[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part_s[threadIdx.x] - sum;  // exclusive
    for (uint32_t j = b0; j < b1; ++j) {
        const uint32_t c = block_counts[j];
        block_counts[j] = run;
        run += c;
    }
    if (threadIdx.x == kScanBlock - 1) *count = part_s[kScanBlock - 1];
}

__global__ __launch_bounds__(kSelBlock) void vit_select_write_kernel(const float* __restrict__ scores,
                                                                     const uint64_t* __restrict__ offsets,
                                                                     const uint32_t* __restrict__ order, uint64_t n,
                                                                     float mu, float lambda, double threshold,
                                                                     const uint32_t* __restrict__ block_prefix,
                                                                     uint32_t* __restrict__ select) {
    __shared__ uint32_t wave_base[4];
    uint32_t idx = 0;
    const uint64_t pos = static_cast<uint64_t>(blockIdx.x) * kSelBlock + threadIdx.x;
    const bool pass = select_pass(scores, offsets, order, n, mu, lambda, threshold, nullptr, pos, &idx);
    const uint64_t mask = __builtin_amdgcn_ballot_w64(pass);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mask >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mask), 0u));
    if (lane == 0) wave_base[wv] = static_cast<uint32_t>(__popcll(mask));
    __syncthreads();
    uint32_t base = block_prefix[blockIdx.x];
    for (uint32_t k = 0; k < wv; ++k) base += wave_base[k];
    if (pass) select[base + below] = idx;
}

hipError_t launch_select(const float* scores, const uint64_t* offsets, const uint32_t* order, uint64_t n, float mu,
                         float lambda, double threshold, double* pvalues, uint32_t* select, uint32_t* count,
                         hipStream_t stream) {
    const uint64_t blocks = (n + kSelBlock - 1) / kSelBlock;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    if (blocks == 0) return hipMemsetAsync(count, 0, sizeof(uint32_t), stream);
    // the per-block counts: stream-ordered scratch, so calls on different streams never share it; a device
    // without memory pools gets a plain allocation, freed after the stream has drained
    int dev = 0, pools = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&pools, hipDeviceAttributeMemoryPoolsSupported, dev);
    if (e != hipSuccess) return e;
    uint32_t* counts = nullptr;
    e = pools ? hipMallocAsync(reinterpret_cast<void**>(&counts), blocks * sizeof(uint32_t), stream)
              : hipMalloc(reinterpret_cast<void**>(&counts), blocks * sizeof(uint32_t));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(vit_select_count_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kSelBlock), 0, stream,
                       scores, offsets, order, n, mu, lambda, threshold, pvalues, counts);
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(vit_select_scan_kernel, dim3(1), dim3(kScanBlock), 0, stream, counts,
                           static_cast<uint32_t>(blocks), count);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(vit_select_write_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kSelBlock), 0, stream,
                           scores, offsets, order, n, mu, lambda, threshold, counts, select);
        e = hipGetLastError();
    }
    hipError_t f;
    if (pools) {
        f = hipFreeAsync(counts, stream);
    } else {
        f = hipStreamSynchronize(stream);
        const hipError_t g = hipFree(counts);
        f = f != hipSuccess ? f : g;
    }
    return e != hipSuccess ? e : f;
}

// ------------------------------------------------------------------------------------------------
// Variant table.  treg + elds: transitions in VGPRs (7 S), match scores in LDS (20 x 64 S floats); the
// compiler holds 10 S + ~30 VGPRs, so up to S = 22 at two waves per SIMD (8 per workgroup).  Beyond,
// transitions move to LDS and match scores are read from L2 every row.  isc variants (insert_mode 1) read
// insert scores from L2 and keep transitions in LDS.
// ------------------------------------------------------------------------------------------------
#define VIT_VARIANT(S_, NT_, ELDS_, ISC_, W_, PD_, ASC_, PICK_, NAME_)                                 \
    VitVariant{S_,                                                                                       \
               NT_,                                                                                      \
               ELDS_,                                                                                    \
               ISC_,                                                                                     \
               W_,                                                                                       \
               PICK_,                                                                                    \
               reinterpret_cast<const void*>(&vit_kernel<S_, NT_, ELDS_, ISC_, W_, PD_, ASC_>),          \
               NAME_,                                                                                    \
               (ELDS_ ? kRows * (S_)*kLanes * 4 : 0) + (kTransitions - (NT_)) * (S_)*kLanes * 4}

// `P` marks the automatic choice per S (interleaved timings on the MSV survivors of cfg3 / cfg5 and on cfg2,
// profiles/r04_vit_tune_cfg{2,3,5}.jsonl); round 5's team variants (vit_team.hip) took over 1,281-1,920 and
// 2,049-2,432 states (profiles/r05_team_tune_bands*.jsonl).  Round 6 pruned the table to the picks, which
// also serve as the fallback of every wider band (set_variant accepts any variant whose S covers the model),
// plus vit_s22_t5a, the single-wave form of the 1,281-1,408 band (the team pick's A/B base).  The ~30 A/B-only
// forms (t5 / t0 splits, descending rows, one wave per SIMD with every transition in VGPRs) are in git history
// up to round 5, with their timings in profiles/r04_vit_tune_*.jsonl.
#define P true
#define X false
static const VitVariant* single_wave_variants(int* count) {
    static const VitVariant all[] = {
        // every transition array in VGPRs, match scores in LDS
        VIT_VARIANT(2, 7, true, false, 8, 0, false, P, "vit_s2_t7"),
        VIT_VARIANT(4, 7, true, false, 8, 0, false, P, "vit_s4_t7"),
        VIT_VARIANT(6, 7, true, false, 8, 0, false, P, "vit_s6_t7"),
        VIT_VARIANT(8, 7, true, false, 8, 0, false, P, "vit_s8_t7"),
        VIT_VARIANT(10, 7, true, false, 8, 0, false, P, "vit_s10_t7"),
        VIT_VARIANT(12, 7, true, false, 8, 0, false, P, "vit_s12_t7"),
        VIT_VARIANT(14, 7, true, false, 8, 0, false, P, "vit_s14_t7"),
        VIT_VARIANT(16, 7, true, false, 8, 0, false, P, "vit_s16_t7"),
        VIT_VARIANT(18, 7, true, false, 8, 0, false, P, "vit_s18_t7"),
        // five arrays in VGPRs (MD, DD in LDS), the row as one ascending pass: cfg3 1.68 vs 1.85 ms at S = 22
        VIT_VARIANT(20, 5, true, false, 8, 1, true, P, "vit_s20_t5a"),
        VIT_VARIANT(22, 5, true, false, 8, 1, true, X, "vit_s22_t5a"),
        // transitions in LDS, match scores from L2 (two waves per SIMD; S = 64 spills, models > 3,072 states only)
        VIT_VARIANT(32, 0, false, false, 8, 3, false, P, "vit_s32_t0g"),
        VIT_VARIANT(64, 0, false, false, 8, 3, false, P, "vit_s64_t0g"),
        // one wave per SIMD (4 per workgroup): the 512-register budget holds S = 48 with 12 spilled VGPRs
        VIT_VARIANT(48, 0, false, false, 4, 3, false, P, "vit_s48_t0g4"),
        // informative insert scores (insert_mode 1): transitions in LDS, match and insert scores from L2
        VIT_VARIANT(2, 0, false, true, 8, 3, false, P, "vit_s2_t0gi"),
        VIT_VARIANT(8, 0, false, true, 8, 3, false, P, "vit_s8_t0gi"),
        VIT_VARIANT(16, 0, false, true, 8, 3, false, P, "vit_s16_t0gi"),
        VIT_VARIANT(22, 0, false, true, 8, 3, false, P, "vit_s22_t0gi"),
        VIT_VARIANT(28, 0, false, true, 8, 3, false, P, "vit_s28_t0gi"),
        VIT_VARIANT(32, 0, false, true, 8, 3, false, P, "vit_s32_t0gi"),
        // ... one wave per SIMD with every transition in VGPRs where two waves spill
        VIT_VARIANT(34, 7, false, true, 4, 3, false, P, "vit_s34_t7gw4i"),
        VIT_VARIANT(38, 7, false, true, 4, 3, false, P, "vit_s38_t7gw4i"),
        VIT_VARIANT(64, 0, false, true, 8, 3, false, P, "vit_s64_t0gi"),
    };
    *count = static_cast<int>(sizeof(all) / sizeof(all[0]));
    return all;
}
#undef P
#undef X

const VitVariant* vit_variants(int* count) {
    static std::vector<VitVariant> all;
    static std::once_flag once;
    std::call_once(once, [] {
        int n1 = 0, n2 = 0;
        const VitVariant* a1 = single_wave_variants(&n1);
        const VitVariant* a2 = vit_team_variants(&n2);
        all.assign(a1, a1 + n1);
        all.insert(all.end(), a2, a2 + n2);
    });
    *count = static_cast<int>(all.size());
    return all.data();
}

hipError_t vit_launch(const VitVariant& v, uint32_t blocks, const VitArgs& args, hipStream_t stream, hipEvent_t start,
                      hipEvent_t stop) {
    void* params[] = {const_cast<VitArgs*>(&args)};
    if (start || stop)
        return hipExtLaunchKernel(v.fn, dim3(blocks), dim3(v.waves * 64), params, 0, stream, start, stop, 0);
    return hipLaunchKernel(v.fn, dim3(blocks), dim3(v.waves * 64), params, 0, stream);
}

}  // namespace vitk
