// msv_kernel.hip -- the MSV hot path as ONE fused CDNA4 (gfx950) kernel per batch.
//
// Replaces MSV_HMM::parallel_run_on_sequence (algorithms/MSV_HMM.cpp:269-430) and its six
// OpenCL kernels (algorithms/MSV_kernels.cl:1-65, MSV_spec_kernels.cl:1-50): the reference
// launches 9-14 kernels PER RESIDUE for ONE sequence; here one persistent launch scores a whole
// batch of sequences against one profile, with every DP row kept on-chip.
//
// Recurrence (bit-exact restatement of MSV_HMM::run_on_sequence, MSV_HMM.cpp:100-112), for a
// residue r at row i:
//     Bt   = B' + tr_B_Mk
//     M_j  = e[r][j] + max(M'_{j-1}, Bt)          j = 1..LENG, M'_0 = -inf
//     E    = max_j M_j
//     J    = max(J' + loop, E + tEJ);  C = max(C' + loop, E + tEC)
//     N    = N' + loop;                B = max(N + move, J + move) == max(N, J) + move
// score = C_L + move.  Only IEEE adds and maxes: max is exact and fl() is monotone, so
// max(N+move, J+move) == fl(max(N,J) + move) bit for bit; no multiply exists, so no contraction.
//
// Mapping (MI355X-first, not a translation of the OpenCL NDRange-per-residue):
//   * A "group" of G lanes (G = 16, 32 or 64; 4/8 for small profiles) owns ONE sequence; lane gl holds the S consecutive
//     match states gl*S+1 .. gl*S+S of the DP row in VGPRs (float M[S]).  A 64-lane wave runs
//     64/G independent sequences.
//   * The j-1 neighbour crosses a lane boundary once per row: one DPP row_shr:1 (+ row_bcast:15
//     for G=32) moves M[S-1] to the next lane; lane 0 of a group reads M_0 = -inf.
//   * E: per-lane max3 tree, then a DPP butterfly (quad_perm, row_half_mirror, row_mirror) and a
//     v_permlane16_swap for G=32 -- no LDS, no barrier.
//   * The 20 x (G*S) fp32 emission table (+1 poison row of +inf for codes >= 20) lives in LDS,
//     laid out [residue][chunk][lane] float4 so every ds_read_b128 of a group is contiguous.
//     One workgroup per CU shares the table across all its waves.  Profiles whose table does not
//     fit the 160 KiB LDS (LENG > ~1920) use the SPLIT layout: each lane's first SA states have all
//     20 rows in LDS, its last S - SA states come from a lane-contiguous global table (L2), read one
//     row ahead as float4; beyond 3072 states the G = 64 row-class layout serves whole rows from LDS
//     or L2 behind a wave-uniform branch.
//   * Persistent grid: every group dequeues sequences from a device counter (prefetched one
//     sequence ahead, one atomic per sequence), so long and short sequences load-balance with no
//     host scheduling; a group that reaches the end of its sequence writes the score and starts
//     the next one in place.
//   * The residue stream is read one byte per row per group (global_load_ubyte, L1/L2-served,
//     1-6 rows of prefetch into rotating slots, by row length); the per-length transition
//     constants come from a host-computed table (host logf, so scores never depend on a device
//     logf).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>
#include <utility>

#include "msv_kernel.h"

namespace msvk {

namespace {

template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ float dpp(float old, float src) {
    // bound_ctrl = false: a lane whose DPP source is invalid keeps `old`.
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, ROW_MASK,
                                                      BANK_MASK, false));
}

constexpr int DPP_QUAD_1032 = 0xB1;    // quad_perm:[1,0,3,2]
constexpr int DPP_QUAD_2301 = 0x4E;    // quad_perm:[2,3,0,1]
constexpr int DPP_ROW_SHR1 = 0x111;    // row_shr:1
constexpr int DPP_ROW_MIRROR = 0x140;  // row_mirror
constexpr int DPP_ROW_HMIRROR = 0x141; // row_half_mirror
constexpr int DPP_ROW_BCAST15 = 0x142; // row_bcast:15

// M_{j-1} for the first state of each lane: the last state of the previous lane of the same
// group; -inf (the dummy M0 column, MSV_HMM.cpp:86) for the first lane of a group.  `old` supplies
// the lanes the shift does not write: -inf there (G < 16: any value, the -inf is selected here).
// For G >= 16 the caller passes the previous result back in, so those lanes keep the -inf written
// once at start and no per-row -inf copy is needed.
template <int G>
__device__ __forceinline__ float shift_in(float last, float old) {
    if constexpr (G < 16) {
        static_assert(G == 4 || G == 8, "G must be 4, 8, 16, 32 or 64");
        const float v = dpp<DPP_ROW_SHR1>(old, last);
        return (threadIdx.x & (G - 1)) == 0 ? -__builtin_inff() : v;  // first lane of each group
    } else if constexpr (G == 16) {
        return dpp<DPP_ROW_SHR1>(old, last);
    } else if constexpr (G == 32) {
        // rows 1 and 3 first receive lane 15 of rows 0 and 2; row_shr:1 then fills every lane
        // except the first of each row, which keeps that broadcast (or -inf for rows 0 and 2).
        float v = dpp<DPP_ROW_BCAST15, 0xA>(old, last);
        return dpp<DPP_ROW_SHR1>(v, last);
    } else {
        static_assert(G == 64, "G must be 16, 32 or 64");
        float v = dpp<DPP_ROW_BCAST15, 0xE>(old, last);  // rows 1-3 get lane 15 of the row before
        return dpp<DPP_ROW_SHR1>(v, last);
    }
}

// In-row permutation (every source lane valid): lets the DPP combiner fold it into v_max_f32_dpp.
template <int CTRL>
__device__ __forceinline__ float dpp_perm(float src) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(src), CTRL, 0xF, 0xF, true));
}

// Lane q of each 16-lane DPP row, broadcast to the whole row (row_newbcast, gfx90a+).
template <int Q>
__device__ __forceinline__ uint32_t row_bcast_lane(uint32_t v) {
    static_assert(Q >= 0 && Q < 16, "row_newbcast lane");
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x150 + Q, 0xF, 0xF, true));
}

// Max over the G lanes of a group, result in every lane of the group.
template <int G>
__device__ __forceinline__ float group_max(float x) {
    x = fmaxf(x, dpp_perm<DPP_QUAD_1032>(x));
    x = fmaxf(x, dpp_perm<DPP_QUAD_2301>(x));
    if constexpr (G >= 8) x = fmaxf(x, dpp_perm<DPP_ROW_HMIRROR>(x));
    if constexpr (G >= 16) x = fmaxf(x, dpp_perm<DPP_ROW_MIRROR>(x));
    if constexpr (G >= 32) {
        auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        x = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
    }
    if constexpr (G == 64) {
        auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        x = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
    }
    return x;
}


template <int G>
__device__ __forceinline__ uint32_t group_bcast(uint32_t v, int lane) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute((lane & ~(G - 1)) << 2, static_cast<int>(v)));
}

// Next sequence index for the whole group (one atomic by the group leader, broadcast).  Indices
// below `first` (the grid's lane groups) are handed out statically: a group's first sequence is its
// own group number, so a wave starts without an atomic round trip.
// Branch-free on purpose: with `if (leader) v = atomicAdd(...)` the ROCm 7.2 optimiser unswitched
// a loop containing this on `leader` into per-lane copies; the non-leader copy lost the atomic and
// its ds_bpermute read a lane that was not executing (a launch that spun forever on index 0).
// Every lane issues the atomic with increment leader ? 1 : 0; the wave-level atomic optimiser turns
// that into one atomic per wave.
template <int G>
__device__ __forceinline__ uint32_t group_take(uint32_t* counter, bool leader, int lane, uint32_t first) {
    const uint32_t v = atomicAdd(counter, leader ? 1u : 0u);
    return group_bcast<G>(v, lane) + first;
}

}  // namespace

// Per-lane state of one sequence being scored (one "stream"): S match states of the DP row in
// VGPRs, the specials, and the residue cursor.  Separate objects (never an indexed array) so all of
// it stays in registers.
// Rows of residue prefetch: a row of a small profile is short (S=8: ~45 VALU), so the byte load
// for a row is issued RPF rows ahead to cover the L2/HBM latency.
template <int S>
constexpr int residue_prefetch() {
    return S <= 16 ? 6 : (S <= 40 ? 3 : 1);
}

// J and C are kept as PER-LANE partials: J_l = max(J_l' + loop, Elane + tEJ) with Elane the max over
// the lane's own states.  Because max is exact and fl() is monotone, max_l J_l equals the
// reference's J = max(J' + loop, E + tEJ) at every row (induction on the row), so the group-wide
// E is never formed per row; the group max is taken only when B needs J (below) and once at the
// end of the sequence for C.
template <int S, int RPF_ = residue_prefetch<S>()>
struct Stream {
    static constexpr int RPF = RPF_;
    float M[S];
    float J, C, N, B, loop, move;
    float nbr;        // M_{j-1} of the lane's first state; lane 0 of each DPP row is never written
                      // by the shift (invalid source), so it keeps the -inf set once at start
    // pos: residue of the current row; endpos: last residue (prefetch clamp); endp: pos after the
    // last row; ev: pos at which the next event fires (the half-way index fetch, then endp)
    uint32_t pos, endpos, endp, ev, seq;
    uint8_t r[RPF];   // residue codes of the next RPF rows (bytes: a 32-bit slot made the compiler
                      // zero-extend each load where it lands, i.e. wait for it in the same row)
    uint32_t cur;     // BLK: residue blocks, lane b of each 16-lane DPP row = the row of phase b
    uint8_t nxt;      // (cur: this 16-row block, clamped to the poison row; nxt: the next one, raw --
                      // a byte for the reason above, so its load is waited for only where it is used)
    bool active;
    bool junk;        // current "sequence" is an empty/too-long record: discard its row
};

// Per-row working set of one stream.
template <int PF>
struct RowCtx {
    static constexpr int kPF = PF;
    const float4* ep;
    float Bt, nbr, p0, p1, p2, p3;  // (p2, p3 unused: keeping them keeps the register assignment measured in round 1)
    uint8_t rnext;   // residue code RPF rows ahead
    float4 ring[PF];
};

// SA > 0 selects the SPLIT layout (G = 32 or 64, tables too large for LDS): lane gl still owns the S
// consecutive states gl*S+1 .. gl*S+S; its first SA states (the "A block") have all 20 residue rows in
// LDS, its last S - SA states (the "B block") are read from the global table (L2) for every row -- no
// per-row LDS/L2 class branch, so the groups of a wave run the same row body whatever their residues;
// the next row's B halves are requested one row ahead.
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0>
__global__ __launch_bounds__(WAVES * 64) void msv_batch_kernel(const KernelArgs a) {
    constexpr bool SPLIT = SA > 0;
    // SPLIT needs the next row's residue one row early (B-chunk prefetch): at least 2 rows.
    using St = Stream<S, (SPLIT && residue_prefetch<S>() < 2) ? 2 : residue_prefetch<S>()>;
    static_assert(SPLIT ? (S - SA) % 2 == 0 : S % 4 == 0, "float4 chunks (A block), float2 halves (B block)");
    static_assert(PF >= 1 && D >= 1 && D <= 2, "PF >= 1, D in {1, 2}");
    static_assert(!SPLIT || (G >= 32 && !BIG && D == 1 && SA % 4 == 0 && SA < S), "split: 32/64-lane groups");
    constexpr int C4 = S / 4;
    constexpr int CA = SPLIT ? SA / 4 : C4;  // float4 chunks per lane whose emissions are staged in LDS
    constexpr int HB = SPLIT ? (S - SA) / 2 : 0;  // SPLIT: float2 halves per lane read from the B table
    constexpr int ROW_F4 = CA * G;           // float4 per LDS residue row
    constexpr int HBP = (HB + 1) & ~1;       // SPLIT: halves per lane in the B table (padded to even)
    constexpr int LDS_ROWS = SPLIT ? kAminoAcids : lds_rows_for(G, S);
    // Residue slots rotate instead of shifting (ROT): the row of phase P reads its residue from
    // r[P] and loads the residue RPF rows ahead into the same slot, and the main loop is unrolled
    // over the RPF phases.  A shift register moves every prefetched byte once per row, and a move of
    // a register with a load in flight waits for that load (s_waitcnt vmcnt(0) in every row): the
    // short rows of small profiles then last as long as one L2 round trip.  Paths that keep the
    // shift: one residue of prefetch (nothing to shift), the G = 64 row-class layout and D = 2.
    constexpr bool ROT = !BIG && D == 1 && St::RPF > 1;
    // Residue BLOCKS (BLK, short rows with G >= 16): instead of one byte load per row, every lane
    // loads one byte of a 16-row block (lane b of each DPP row: the row of phase b), once per 16
    // rows, a block ahead; a row takes its residue with one row_newbcast DPP move.  The row loop is
    // unrolled over the 16 phases and the block in flight is consumed 14-16 rows after its load, so
    // the waits the compiler places at the loop header or after a rare path (which merge every load
    // in flight: with per-row slots the header waited for the load of the row before, once per RPF
    // rows -- the bound of cfg2's 100.hmm rows) find it landed.  16x fewer VMEM instructions.
#ifndef MSV_BLK_LARGE
#define MSV_BLK_LARGE 0
#endif
    // rows per block: 16 for short rows; long rows (one residue of prefetch) optionally 8 (experiment)
    constexpr int BLKN = St::RPF > 1 ? 16 : MSV_BLK_LARGE;
    constexpr bool BLK = !BIG && D == 1 && G >= 16 && !SPLIT && BLKN > 0;
    constexpr int NPH = BLK ? BLKN : St::RPF;  // phases of the unrolled row loop
    // Cross-row emission prefetch: when the ring holds a whole row (small profiles), the NEXT row's
    // chunks are requested right after this row's last cell update, so the LDS latency hides behind
    // the E butterfly and the specials instead of stalling the start of every row.
    constexpr bool XROW = !BIG && !SPLIT && D == 1 && PF >= C4 && St::RPF >= 2;
    // ... and two rows ahead when the residue slots rotate over an even number of phases: rows of
    // even and odd phase keep their own ring, refilled with the row after next right after use, so
    // the LDS reads have a whole row to land instead of the epilogue's dozen instructions (cfg2:
    // 100.hmm rows are ~35 VALU, and waves spent 67% of their cycles in s_waitcnt, PMC r02).
#ifndef MSV_XROW_DEPTH
#define MSV_XROW_DEPTH 2
#endif
    constexpr bool XROW2 = XROW && MSV_XROW_DEPTH == 2 && NPH % 2 == 0 && PF <= 2;  // +4 PF VGPRs
    static_assert(SPLIT || BIG == (LDS_ROWS < kTableRows), "BIG <=> table does not fit LDS");
    __shared__ float4 tab[LDS_ROWS * ROW_F4];

    const float NINF = -__builtin_inff();
    const int lane = threadIdx.x & 63;
    const int gl = lane & (G - 1);
    const bool leader = gl == 0;

    // Stage the emission table (already in kernel layout) into LDS once per workgroup.
    for (int i = threadIdx.x; i < LDS_ROWS * ROW_F4; i += WAVES * 64) tab[i] = a.etab[i];
    __syncthreads();

    const uint8_t* __restrict__ res = a.residues;
    const float trBMk = a.tr_B_Mk, tEC = a.tr_E_C, tEJ = a.tr_E_J;
    const bool sameEJ = __float_as_uint(tEC) == __float_as_uint(tEJ);  // wave-uniform (SGPR)

    uint32_t rows_done = 0;  // rows issued by this wave (diagnostics)
    // Work distribution: a group's first sequence is its group number; the index of its next sequence
    // is fetched while the current one runs.  Long rows (S >= 64) fetch it 8 + 256/S rows before the
    // end -- enough to hide the atomic's round trip, late enough that the last indices go to the
    // groups actually about to finish rather than to every group half-way through its sequence:
    // cfg5 25.50 -> 25.03 ms, cfg3 neutral.  Short rows fetch half-way: their sequences end ~100 per
    // us, and at that rate the one counter's atomics queue for more than 17 rows of 28 states
    // (400.hmm x 100k: 1.034 vs 1.004 ms late; profiles/r02_ab_fetch_ahead.jsonl).
#ifndef MSV_FETCH_AHEAD
#define MSV_FETCH_AHEAD (S >= 64 ? 8 + 256 / S : 0xFFFFFFFFu)
#endif
    constexpr uint32_t kFetchAhead = MSV_FETCH_AHEAD;
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    const uint32_t n_groups = gridDim.x * (WAVES * 64 / G);  // statically assigned first indices
    // The group's first sequence (the first stream's begin consumes it).  With the longest-first order,
    // neighbouring indices have similar lengths.  Wave w of a block runs on SIMD (w mod 4), so the block's
    // waves are dealt in rounds of 4 (one per SIMD): wave w of block b takes the wave-set (64/G
    // consecutive indices) r * 4 * gridDim.x + 4 * b + (w mod 4), r = w / 4.  The groups of a wave and
    // the 4 SIMDs of a round get similar lengths; successive rounds (the waves sharing a SIMD) come from
    // different parts of the order.  (Block b taking indices [b * groups, ...) gave the 16 waves of a
    // 64-lane-plan block, 4 per SIMD, the 16 longest sequences of the batch: 1400.hmm x 8192 0.66 vs
    // 0.46 ms, 1901.hmm x 256 0.44 vs 0.26 ms; dealing single groups over blocks put each block's
    // longest sequences on one SIMD: cfg2 0.105 vs 0.185 ms -- profiles/r02_ab_first_assignment.jsonl.)
    // Batches larger than the grid (the counter hands out the rest) keep block b on indices [b * groups,
    // ...): there the first sequences all have about the same length, and the rounds measured 0.4-1%
    // slower on cfg3/cfg5.
    static_assert(WAVES % 4 == 0, "waves are dealt in rounds of one per SIMD");
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t wave_set = a.n <= n_groups ? (wave >> 2) * 4u * gridDim.x + 4u * blockIdx.x + (wave & 3u)
                                              : blockIdx.x * WAVES + wave;
    uint32_t pending = wave_set * (64 / G) + static_cast<uint32_t>(lane / G);

#ifndef MSV_YOUNG_CUTOFF
#define MSV_YOUNG_CUTOFF 8
#endif
    // Drain tail.  The waves of a block are arbitrated oldest-first on their SIMD, so the youngest
    // quarter issue last: a sequence they take near the end of the queue finishes last and sets the
    // launch's end (cfg3 timeline: waves 12-15 did a fifth of the rows of waves 0-3 and still ended
    // 90 us after them -- profiles/r02_wave_timeline_cfg3.jsonl).  For large profiles (S >= 64, whose
    // rows are long enough that fewer waves still keep the SIMD issuing) those waves stop taking
    // sequences once fewer than n_groups * MSV_YOUNG_CUTOFF / 4 remain and leave them to the older
    // waves: cfg3 2.93 -> 2.88 ms, the other large profiles within 0.3%.  Small profiles stay
    // issue-bound to the end (cfg2 lost 9%), so they keep every wave -- profiles/r02_ab_young_cutoff.jsonl.
    constexpr uint32_t kYoung = S >= 64 ? MSV_YOUNG_CUTOFF : 0;
    const bool young = kYoung > 0 && (threadIdx.x >> 6) >= (3u * WAVES) / 4u;
    auto take = [&]() __attribute__((always_inline)) -> uint32_t {
        if constexpr (kYoung > 0) {
            if (young) {
                const uint32_t cur = group_take<G>(a.counter, false, lane, n_groups);  // +0: a read
                if (static_cast<uint64_t>(cur) + (static_cast<uint64_t>(n_groups) * kYoung) / 4 >= a.n)
                    return 0xFFFFFFFEu;  // >= n: retire
            }
        }
        return group_take<G>(a.counter, leader, lane, n_groups);
    };
    using Ph0 = std::integral_constant<int, 0>;
    const uint32_t blk_lane = static_cast<uint32_t>(gl & (BLKN > 0 ? BLKN - 1 : 0));  // BLK: the lane's row in a block

    // Start the next non-empty sequence in a stream (or retire the stream); `ph` is the phase of the
    // row that will run next (its residue goes to slot r[ph]).
    auto begin = [&](St& st, auto ph) __attribute__((always_inline)) {
        constexpr int PH = decltype(ph)::value;
        // Loop-free on purpose: a retry loop around the group broadcast here was unswitched by
        // the compiler into per-lane copies (see group_take).  An empty (or too long) record
        // instead becomes a one-row "junk" stream: its score is written now, one row is computed
        // on neutral state and discarded, and the stream then restarts with the next index.
        uint32_t idx = pending;
        pending = kNone;
        if (idx == kNone) idx = take();
        const bool retire = idx >= a.n;
        uint32_t s = 0;
        uint64_t o0 = 0, o1 = 0;
        if (!retire) {
            s = a.order ? a.order[idx] : idx;
            o0 = a.offsets[s];
            o1 = a.offsets[s + 1];
        }
        const uint64_t L = o1 - o0;
        const bool empty = !retire && L == 0;            // C_0 = -inf (MSV_HMM.cpp:86,112)
        const bool too_long = !retire && L >= a.lentab_n;
        if (leader && empty) a.scores[s] = NINF;
        if (leader && too_long) {
            a.scores[s] = __uint_as_float(0x7fc00000u);  // quiet NaN bits
            atomicOr(a.errors, kErrTooLong);
        }
        const bool run = !retire && !empty && !too_long;
        // A retired or junk stream runs with move = -inf: B = Bt = -inf keeps its rows at -inf, so
        // its J partials never reach N and never force the epilogue's group reduction.
        const float2 lm = run ? a.lentab[L] : make_float2(0.f, NINF);
        st.loop = lm.x;
        st.move = lm.y;
        st.seq = s;
        st.pos = run ? static_cast<uint32_t>(o0) : 0u;
        st.endpos = run ? static_cast<uint32_t>(o1 - 1) : 0u;
        // a junk stream ends after its one row; a retired one never (pos cannot reach 2^32 - 1)
        st.endp = retire ? 0xFFFFFFFFu : (run ? static_cast<uint32_t>(o1) : 1u);
        // the next index is fetched kFetchAhead rows before the end (half-way for shorter sequences;
        // equal to endp when L == 1: begin fetches it)
        st.ev = run ? static_cast<uint32_t>(o1 - min(L >> 1, static_cast<uint64_t>(kFetchAhead))) : st.endp;
#pragma unroll
        for (int k = 0; k < S; ++k) st.M[k] = NINF;
        st.J = NINF;
        st.C = NINF;
        st.N = 0.f;       // dp[0][N] = 0      (MSV_HMM.cpp:96)
        st.B = st.move;   // dp[0][B] = tr_move (MSV_HMM.cpp:97)
        st.active = !retire;
        st.junk = !run;
        if constexpr (BLK) {
            // The first row runs at phase PH: cur lane b (b >= PH) = residue pos + b - PH, nxt lane b =
            // pos + 16 + b - PH.  PH = 0: the phase-0 row first moves nxt into cur, so both hold the
            // first block.  (Lanes below PH are never read; max() keeps their index >= pos.)
            const uint32_t ic = max(st.pos + blk_lane, st.pos + PH) - PH;
            const uint32_t in = PH == 0 ? ic : st.pos + blk_lane + (BLKN - PH);
            st.cur = min(static_cast<uint32_t>(res[min(ic, st.endpos)]), static_cast<uint32_t>(kPoisonRow));
            st.nxt = res[min(in, st.endpos)];
        } else {
#pragma unroll
            for (int q = 0; q < St::RPF; ++q) st.r[(PH + q) % St::RPF] = res[min(st.pos + q, st.endpos)];
        }
    };
    // Residue code of the row at phase P (0 <= P < NPH + 2) for a row of phase <= P: BLK reads it from
    // the blocks (clamped to the poison row); otherwise the slot (clamped where the row address is made).
    auto resid = [&](St& st, auto pp) __attribute__((always_inline)) -> uint32_t {
        constexpr int P = decltype(pp)::value;
        if constexpr (BLK) {
            if constexpr (P < BLKN) {
                return row_bcast_lane<P>(st.cur);
            } else {
                return min(row_bcast_lane<P - BLKN>(static_cast<uint32_t>(st.nxt)), static_cast<uint32_t>(kPoisonRow));
            }
        } else {
            return st.r[P % St::RPF];
        }
    };
    auto init = [&](St& st) {
        st.nbr = NINF;
        begin(st, Ph0{});
    };
    // Row prologue: next residue prefetch, emission row pointer, Bt, the j-1 neighbour, ring fill.
    // LDS row of residue code r for this lane (codes >= 20 -> the poison row).  (A hand-written
    // v_min_sdwa + v_mad_u32_u24 form of this address, and pinning the prefetched residue as a
    // 32-bit value, each measured 2-4% slower on 1400.hmm: they move the residue-load wait.)
    // (SPLIT: the LDS holds rows 0..19 only; codes >= 20 read row 19 there and the +inf poison row
    // of the B table, which still makes the score +inf.)
    // The address is one v_mad_u32_u24 on a hoisted lane byte offset (the index form
    // rr * ROW_F4 + gl compiled to v_mul_u32_u24 + v_or: profiles/r01_ab_row_address.jsonl).
    const uint32_t lds_lane = static_cast<uint32_t>(gl * 16);
    auto lds_row = [&](uint32_t r) -> const float4* {
        // (BLK residues arrive clamped)
        const uint32_t rr = BLK ? r : min(r, static_cast<uint32_t>(SPLIT ? kAminoAcids - 1 : kPoisonRow));
        uint32_t off;
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(off) : "v"(rr), "s"(static_cast<uint32_t>(ROW_F4 * 16)), "v"(lds_lane));
        return reinterpret_cast<const float4*>(reinterpret_cast<const char*>(tab) + off);
    };
    // SPLIT: the B table ([21][G][HBP] float2: 2-state halves, so the padding past LENG stays under
    // 2 states per lane; lane-contiguous, read as float4) follows the 20 LDS rows in a.etab; the
    // current row's B halves live in `bring`, requested one row ahead.
    const float2* __restrict__ etabB = reinterpret_cast<const float2*>(a.etab + kAminoAcids * ROW_F4);
    struct BRing {
        float2 v[HB > 0 ? HB : 1];
    } bring;
    const uint32_t b_lane = static_cast<uint32_t>(gl * HBP * 8);  // SPLIT: the lane's B halves, in bytes
    auto fill_b = [&](uint32_t r) {
        if constexpr (SPLIT) {
            // lane-contiguous halves: HBP/2 float4 loads per lane (half the VMEM issues of float2 loads
            // strided by G: cfg5 25.08 vs 25.56 ms, profiles/r01_exp_split_b.jsonl)
            // byte offset = row * (G * HBP * 8) + the lane's hoisted offset: one v_mad_u32_u24
            const uint32_t off = min(r, static_cast<uint32_t>(kPoisonRow)) * static_cast<uint32_t>(G * HBP * 8) + b_lane;
            const float4* bp = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(etabB) + off);
#pragma unroll
            for (int q = 0; q < HBP / 2; ++q) {
                const float4 v = bp[q];
                bring.v[2 * q] = make_float2(v.x, v.y);
                if (2 * q + 1 < HB) bring.v[2 * q + 1] = make_float2(v.z, v.w);
            }
        }
    };
    auto row_ptr = [&](St& st, auto ph) -> const float4* {
        if constexpr (!BIG) {
            return lds_row(resid(st, ph));
        } else {
            const uint32_t rr = min(st.r[0], static_cast<uint32_t>(kPoisonRow));
            return (rr < static_cast<uint32_t>(LDS_ROWS)) ? &tab[rr * ROW_F4 + gl] : &a.etab[rr * ROW_F4 + gl];
        }
    };
    // Request the first chunks of a row (all of it when the ring holds a whole row).
    auto fill_ring = [&](auto& rc, const float4* ep) {
        constexpr int P = std::decay_t<decltype(rc)>::kPF;
#pragma unroll
        for (int q = 0; q < (P < CA ? P : CA); ++q) rc.ring[q] = ep[(CA - 1 - q) * G];
    };
    auto prologue = [&](St& st, auto& rc, const float4* ep, auto ph) {
        (void)ph;
        if constexpr (!BLK) rc.rnext = res[min(st.pos + St::RPF, st.endpos)];
        rc.ep = ep;
        rc.Bt = st.B + trBMk;
        if constexpr (G >= 16) {
            st.nbr = shift_in<G>(st.M[S - 1], st.nbr);
            rc.nbr = st.nbr;
        } else {
            rc.nbr = shift_in<G>(st.M[S - 1], NINF);
        }
        // p0/p1 start from the row's first chunk (a plain max, no -inf seed)
        if constexpr (!XROW) fill_ring(rc, ep);
    };
    // One float4 chunk (states 4c+1 .. 4c+4 of the lane), highest state first so M[k-1] is still
    // the previous row's value; the next chunk is requested PF chunks ahead.
    auto chunk = [&](St& st, auto& rc, auto cc) {
        constexpr int P = std::decay_t<decltype(rc)>::kPF;
        constexpr int c = decltype(cc)::value;
        constexpr int slot = (CA - 1 - c) % P;
        const float4 ev = rc.ring[slot];
        if constexpr (c - P >= 0) rc.ring[slot] = rc.ep[(c - P) * G];
        constexpr int k = 4 * c;
        if constexpr (!BIG && S >= 64) {
            // The chunk's 10 VALU ops in a fixed interleaved order (max, max, add, max, add, max, add,
            // max3, add, max3).  gfx950 issues v_max/v_max3 at half the v_add rate and overlaps the two
            // kinds when they alternate; in isolation the compiler's grouping ([4 max][4 add][2 max3])
            // runs 17.2-18.0 cells/ns/SIMD against 20.0-21.0 for this order (tools/micro/row_sched.hip).
            // Inside the kernel the per-row work and LDS traffic fill most of the grouping's gaps: +1.4%
            // on 1400.hmm (2.924 vs 2.964 ms, interleaved A/B), and slower for small rows and for the
            // G = 64 BIG rows (9.2 vs 7.2 ms), which keep the compiler's schedule.
            // Same IEEE ops as the C++ below: max is exact, so max3(p, a, b) == max(max(p, a), b).
            const float mprev = c == 0 ? rc.nbr : st.M[k > 0 ? k - 1 : 0];
            // first two maxes need no emission: a separate block, so the wait for the chunk's LDS
            // data lands after them
            asm volatile(
                "v_max_f32 %0, %1, %4\n\t"
                "v_max_f32 %1, %2, %4"
                : "+v"(st.M[k + 3]), "+v"(st.M[k + 2]), "+v"(st.M[k + 1])
                : "v"(st.M[k]), "v"(rc.Bt));
            if constexpr (!SPLIT && c == CA - 1) {  // the row's first chunk starts the E partials
                asm volatile(
                    "v_add_f32 %0, %8, %0\n\t"
                    "v_max_f32 %2, %3, %7\n\t"
                    "v_add_f32 %1, %9, %1\n\t"
                    "v_max_f32 %3, %6, %7\n\t"
                    "v_add_f32 %2, %10, %2\n\t"
                    "v_max_f32 %4, %0, %1\n\t"
                    "v_add_f32 %3, %11, %3\n\t"
                    "v_max_f32 %5, %2, %3"
                    : "+v"(st.M[k + 3]), "+v"(st.M[k + 2]), "+v"(st.M[k + 1]), "+v"(st.M[k]), "=&v"(rc.p0),
                      "=&v"(rc.p1)
                    : "v"(mprev), "v"(rc.Bt), "v"(ev.w), "v"(ev.z), "v"(ev.y), "v"(ev.x));
            } else {
                asm volatile(
                    "v_add_f32 %0, %8, %0\n\t"
                    "v_max_f32 %2, %3, %7\n\t"
                    "v_add_f32 %1, %9, %1\n\t"
                    "v_max_f32 %3, %6, %7\n\t"
                    "v_add_f32 %2, %10, %2\n\t"
                    "v_max3_f32 %4, %4, %0, %1\n\t"
                    "v_add_f32 %3, %11, %3\n\t"
                    "v_max3_f32 %5, %5, %2, %3"
                    : "+v"(st.M[k + 3]), "+v"(st.M[k + 2]), "+v"(st.M[k + 1]), "+v"(st.M[k]), "+v"(rc.p0),
                      "+v"(rc.p1)
                    : "v"(mprev), "v"(rc.Bt), "v"(ev.w), "v"(ev.z), "v"(ev.y), "v"(ev.x));
            }
            return;
        }
        // small rows and BIG rows: the compiler-scheduled form of the same chunk
        st.M[k + 3] = ev.w + fmaxf(st.M[k + 2], rc.Bt);
        st.M[k + 2] = ev.z + fmaxf(st.M[k + 1], rc.Bt);
        st.M[k + 1] = ev.y + fmaxf(st.M[k], rc.Bt);
        if constexpr (c == 0) {
            st.M[k] = ev.x + fmaxf(rc.nbr, rc.Bt);
        } else {
            st.M[k] = ev.x + fmaxf(st.M[k - 1], rc.Bt);
        }
        if constexpr (!SPLIT && c == CA - 1) {  // the row's first chunk: no -inf seed
            rc.p0 = fmaxf(st.M[k + 3], st.M[k + 2]);
            rc.p1 = fmaxf(st.M[k + 1], st.M[k]);
        } else {
            rc.p0 = fmaxf(fmaxf(rc.p0, st.M[k + 3]), st.M[k + 2]);
            rc.p1 = fmaxf(fmaxf(rc.p1, st.M[k + 1]), st.M[k]);
        }
    };
    // SPLIT: one B half (states SA + 2h + 1, + 2 of the lane), emissions already in registers;
    // processed before the A chunks (higher states first, so M[SA - 1] is still the previous row's),
    // the first one seeds the E partials.
    auto bhalf = [&](St& st, auto& rc, auto hh) {
        constexpr int h = decltype(hh)::value;
        constexpr int k = SA + 2 * h;
        const float2 ev = bring.v[h];
        st.M[k + 1] = ev.y + fmaxf(st.M[k], rc.Bt);
        st.M[k] = ev.x + fmaxf(st.M[k - 1], rc.Bt);
        if constexpr (h == HB - 1) {
            rc.p0 = fmaxf(st.M[k + 1], st.M[k]);
            if constexpr (HB == 1) rc.p1 = NINF;
        } else if constexpr (h == HB - 2) {
            rc.p1 = fmaxf(st.M[k + 1], st.M[k]);
        } else if constexpr ((HB - 1 - h) & 1) {
            rc.p1 = fmaxf(fmaxf(rc.p1, st.M[k + 1]), st.M[k]);
        } else {
            rc.p0 = fmaxf(fmaxf(rc.p0, st.M[k + 1]), st.M[k]);
        }
    };
    // Row epilogue: E over the group, the specials (MSV_HMM.cpp:107-110), cursor advance.
    auto epilogue = [&](St& st, auto& rc, auto ph) {
        const float Elane = fmaxf(rc.p0, rc.p1);
        // Per-lane partials (see Stream): J_l, and C_l unless C == J (tr_E_C == tr_E_J, which is
        // always the case for the reference's nu = 2, MSV_HMM.cpp:49-53: then the C and J
        // recurrences are identical and C is read from J at the end).
        const float EJ = Elane + tEJ;
        st.J = fmaxf(st.J + st.loop, EJ);
        if (__builtin_expect(!sameEJ, 0)) {
            st.C = fmaxf(st.C + st.loop, Elane + tEC);
            asm volatile("" ::: "memory");  // keep a real (scalar) branch, not a per-row select
        }
        st.N = st.N + st.loop;
        // B = max(N, J) + move needs the group's J = max_l J_l only if some J_l >= N; otherwise
        // max(N, J) == N exactly.  On random-like sequences J stays below N, so the per-row E/J
        // reduction across lanes (DPP butterfly) leaves the row's dependency chain.
        // (G = 64: a row_bcast:15/31 + v_readlane reduction to an SGPR measured 13% slower on
        // 2405.hmm than the permlane swaps -- the SGPR round trip stalls the row)
        // The common value first and the rare one as an overwrite, so the common path falls through
        // (as an if/else the else-block was laid out of line: two taken branches per row).  The test
        // and branch cost 6% of the cfg2 kernel, 0.5% of cfg3 (profiles/r01_exp_speculative_b.jsonl).
        st.B = st.N + st.move;
        if (__builtin_expect(__any(st.J >= st.N), 0)) st.B = fmaxf(st.N, group_max<G>(st.J)) + st.move;
        ++st.pos;
        if constexpr (BLK) {
            // the blocks advance once per 16 rows (step, phase 0)
        } else if constexpr (ROT) {
            st.r[decltype(ph)::value] = rc.rnext;  // this row's slot now holds the row RPF ahead
        } else {
#pragma unroll
            for (int q = 0; q + 1 < St::RPF; ++q) st.r[q] = st.r[q + 1];
            st.r[St::RPF - 1] = rc.rnext;
        }
    };
    // `ph`: phase of the row that runs next.
    auto finish = [&](St& st, auto ph) __attribute__((always_inline)) {
        // Every lane of the group is here (pos == endp is group-uniform), so the group reduction of
        // the C partials reads only active lanes of the same group.
        // (the copy of J is opaque so the compiler cannot hoist this select into every row)
        float csrc = st.C;
        if (sameEJ) asm volatile("v_mov_b32 %0, %1" : "=v"(csrc) : "v"(st.J));
        const float C = group_max<G>(csrc);
        const float sc = C + st.move;  // dp.back()[C] + tr_move (MSV_HMM.cpp:112)
        if (leader && !st.junk) {
            a.scores[st.seq] = sc;
            if (!(sc <= 3.402823466e38f)) atomicOr(a.errors, kErrBadResidue);  // poison row hit
        }
        begin(st, ph);
    };

    // D independent sequences per lane group ("streams"): their rows interleave chunk by chunk,
    // so one stream's serial per-row section (E butterfly -> J/C/N/B -> Bt) overlaps the other
    // stream's cell updates inside the same wave.
    St s0, s1;
    init(s0);
    if constexpr (D == 2) init(s1);

    uint64_t t_start = 0;
    if (a.stamps) t_start = __builtin_amdgcn_s_memrealtime();

    // (Branch-layout hints -- __builtin_expect on the rare end-of-sequence / prefetch events, or on
    // the LDS-row class for G = 64 -- measured no gain, and 15% LOSS for the latter on 2405.hmm.)

    RowCtx<PF> xr, xr1;  // XROW: the ring persists across rows (XROW2: xr for even phases, xr1 for odd)
    if constexpr (XROW) fill_ring(xr, row_ptr(s0, Ph0{}));
    if constexpr (XROW2) fill_ring(xr1, lds_row(resid(s0, std::integral_constant<int, 1>{})));
    fill_b(s0.r[0]);

    // slot of the residue of the row after a row of phase P
    auto next_slot = [](auto ph) { return (decltype(ph)::value + 1) % St::RPF; };

    // All chunks of one row, C4-1 .. 0, each step pinned so only the rings' registers are live.
    auto row = [&](St& st, auto& rc, const float4* ep, auto ph) {
        prologue(st, rc, ep, ph);
        if constexpr (SPLIT) {
            [&]<int... I>(std::integer_sequence<int, I...>) {
                ((bhalf(st, rc, std::integral_constant<int, HB - 1 - I>{}),
                  [&] { if constexpr (I & 1) __builtin_amdgcn_sched_barrier(0); }()),
                 ...);
            }(std::make_integer_sequence<int, HB>{});
            fill_b(st.r[next_slot(ph)]);  // this row's B halves are consumed: request the next row's
            __builtin_amdgcn_sched_barrier(0);
        }
        [&]<int... I>(std::integer_sequence<int, I...>) {
            ((chunk(st, rc, std::integral_constant<int, CA - 1 - I>{}), __builtin_amdgcn_sched_barrier(0)), ...);
        }(std::make_integer_sequence<int, CA>{});
        epilogue(st, rc, ph);
    };

    // Wave-uniform loop condition, refreshed only when a stream finishes.
    bool live = __any(D == 2 ? (s0.active || s1.active) : s0.active);

    // One row of phase P of the single-stream, non-row-class paths (XROW or plain), then its events.
    // Returns whether the wave still has work.
    auto step = [&](auto ph) __attribute__((always_inline)) -> bool {  // always_inline: 16 BLK phases exceed the inliner's budget
        constexpr int PH = decltype(ph)::value;
        constexpr int PN = (PH + 1) % NPH;
        using PhN = std::integral_constant<int, PN>;
        if constexpr (BLK && PH == 0) {
            // a new 16-row block: the one loaded 16 rows ago becomes current, the next is requested
            s0.cur = min(static_cast<uint32_t>(s0.nxt), static_cast<uint32_t>(kPoisonRow));
            s0.nxt = res[min(s0.pos + BLKN + blk_lane, s0.endpos)];
        }
        if constexpr (XROW2) {
            RowCtx<PF>& rc = (PH & 1) ? xr1 : xr;
            prologue(s0, rc, nullptr, ph);
            [&]<int... I>(std::integer_sequence<int, I...>) {
                ((chunk(s0, rc, std::integral_constant<int, C4 - 1 - I>{})), ...);
            }(std::make_integer_sequence<int, C4>{});
            // the residue of the row after next (discarded if the sequence ends first)
            fill_ring(rc, lds_row(resid(s0, std::integral_constant<int, PH + 2>{})));
            epilogue(s0, rc, ph);
        } else if constexpr (XROW) {
            prologue(s0, xr, nullptr, ph);
            [&]<int... I>(std::integer_sequence<int, I...>) {
                ((chunk(s0, xr, std::integral_constant<int, C4 - 1 - I>{})), ...);
            }(std::make_integer_sequence<int, C4>{});
            // the residue of the next row (discarded if this row ends the sequence)
            fill_ring(xr, lds_row(resid(s0, std::integral_constant<int, PH + 1>{})));
            epilogue(s0, xr, ph);
        } else {
            RowCtx<PF> c0;
            row(s0, c0, row_ptr(s0, ph), ph);
        }
        // Events: see the generic loop below.
        if (G == 64 || __any(s0.pos == s0.ev)) {
            if (s0.pos == s0.ev && s0.ev != s0.endp) {
                if (pending == kNone) pending = take();
                s0.ev = s0.endp;
            }
            if (s0.pos == s0.endp) {
                finish(s0, PhN{});
                if constexpr (XROW2) {  // the new sequence's first two rows
                    fill_ring((PN & 1) ? xr1 : xr, row_ptr(s0, PhN{}));
                    fill_ring((PN & 1) ? xr : xr1, lds_row(resid(s0, std::integral_constant<int, PN + 1>{})));
                } else if constexpr (XROW) {
                    fill_ring(xr, row_ptr(s0, PhN{}));
                }
                if constexpr (SPLIT) fill_b(s0.r[PN]);
            }
            live = __any(s0.active);
        }
        ++rows_done;
        return live;
    };

    while (live) {
        if constexpr (ROT || BLK) {
            // NPH rows per iteration (residue slots, or the 16 rows of a BLK block); stops after any row that retires the wave
            [&]<int... I>(std::integer_sequence<int, I...>) {
                (void)(step(std::integral_constant<int, I>{}) && ...);
            }(std::make_integer_sequence<int, NPH>{});
        } else {
            if constexpr (BIG && G == 64) {
                // One sequence per wave: the residue, hence the table row's home, is wave-uniform, so
                // the LDS rows and the L2 rows run as two separate (scalar-branched) row bodies with
                // precise waits -- no generic loads, no per-lane selects.  An L2 row requests up to 10
                // chunks up front to pay the L2 latency about once per row.
                // (a vector compare with exec masking instead of readfirstlane measured 1.5% slower;
                // reading the class one row early into an SGPR changed nothing; a timing-only form
                // with no class branch at all, wrong scores, ran the row 10% faster)
                const uint32_t rr =
                    __builtin_amdgcn_readfirstlane(min(s0.r[0], static_cast<uint32_t>(kPoisonRow)));
                if (rr < static_cast<uint32_t>(LDS_ROWS)) {
                    RowCtx<PF> c0;
                    row(s0, c0, &tab[rr * ROW_F4 + gl], Ph0{});
                } else {
                    RowCtx<(C4 < 10 ? C4 : 10)> c0;
                    row(s0, c0, &a.etab[rr * ROW_F4 + gl], Ph0{});
                }
            } else if constexpr (D == 1) {
                RowCtx<PF> c0;
                row(s0, c0, row_ptr(s0, Ph0{}), Ph0{});
            } else {
                RowCtx<PF> c0, c1;
                prologue(s0, c0, row_ptr(s0, Ph0{}), Ph0{});
                prologue(s1, c1, row_ptr(s1, Ph0{}), Ph0{});
                [&]<int... I>(std::integer_sequence<int, I...>) {
                    ((chunk(s0, c0, std::integral_constant<int, C4 - 1 - I>{}),
                      chunk(s1, c1, std::integral_constant<int, C4 - 1 - I>{}), __builtin_amdgcn_sched_barrier(0)),
                     ...);
                }(std::make_integer_sequence<int, C4>{});
                epilogue(s0, c0, Ph0{});
                epilogue(s1, c1, Ph0{});
            }
            // Events (one compare per stream and row; the handling is rare and wave-uniformly
            // skipped): the half-way fetch of the next index, then the end of the sequence.  (G = 64:
            // the cursor is wave-uniform and the compares are scalar; there the guard made the
            // compiler copy the whole DP row at the loop latch, +12% per row on 2405.hmm, so it is
            // left out.)
            if (G == 64 || __any(D == 2 ? (s0.pos == s0.ev || s1.pos == s1.ev) : s0.pos == s0.ev)) {
                if (s0.pos == s0.ev && s0.ev != s0.endp) {
                    if (pending == kNone) pending = take();
                    s0.ev = s0.endp;
                }
                if constexpr (D == 2) {
                    if (s1.pos == s1.ev && s1.ev != s1.endp) {
                        if (pending == kNone) pending = take();
                        s1.ev = s1.endp;
                    }
                }
                if (s0.pos == s0.endp) {
                    finish(s0, Ph0{});
                    fill_b(s0.r[0]);
                }
                if constexpr (D == 2) {
                    if (s1.pos == s1.endp) finish(s1, Ph0{});
                }
                live = __any(D == 2 ? (s0.active || s1.active) : s0.active);
            }
            ++rows_done;
        }
    }
    // Self-resetting dequeue counter: the last wave of the grid to leave puts counter[0] (next
    // index) and counter[1] (waves left) back to 0, so the next launch needs no memset.  Every
    // wave's last dequeue atomic has returned before its exit increment.
    if (lane == 0) {
        const uint32_t total = gridDim.x * WAVES;
        if (atomicAdd(a.counter + 1, 1u) == total - 1) {
            atomicExch(a.counter, 0u);
            atomicExch(a.counter + 1, 0u);
        }
    }
    // Diagnostic only (a.stamps == nullptr in production): per-wave start/end realtime (100 MHz),
    // rows issued, XCC id.  Never read by the kernel; used by tools/wave_timeline.py.
    if (a.stamps && lane == 0) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const uint32_t w = blockIdx.x * WAVES + (threadIdx.x >> 6);
        uint32_t xcc = 0, hwid = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        a.stamps[4 * w + 0] = t_start;
        a.stamps[4 * w + 1] = t_end;
        a.stamps[4 * w + 2] = (static_cast<uint64_t>(hwid) << 32) | rows_done;
        a.stamps[4 * w + 3] = (static_cast<uint64_t>(xcc) << 32) | blockIdx.x;
    }
}

// ------------------------------------------------------------------------------------------------
// Longest-first dequeue order: a device counting sort on sequence length (lengths >= nbins-1 share
// the first bin).  Three small launches, histograms privatised in LDS so global atomics are one
// per (block, non-empty bin):  count -> scan -> place.  Order inside a bin is arbitrary (it never
// changes a score: every score is written to its own sequence's slot).  The scratch is [hist |
// cursor]: the scan writes the cursors and zeroes the histogram for the next sort, so no memset
// launch precedes a sort (the caller zeroes a fresh or failed scratch once).
// ------------------------------------------------------------------------------------------------
constexpr int kOrderThreads = 1024;

__device__ __forceinline__ uint32_t length_bin(const uint64_t* __restrict__ offsets, uint64_t s, uint32_t nbins) {
    const uint64_t L = offsets[s + 1] - offsets[s];
    return nbins - 1 - static_cast<uint32_t>(L >= nbins - 1 ? nbins - 1 : L);  // descending length
}

__global__ __launch_bounds__(kOrderThreads) void order_count_kernel(const uint64_t* __restrict__ offsets, uint64_t n,
                                                                    uint64_t chunk, uint32_t* __restrict__ hist,
                                                                    uint32_t nbins) {
    extern __shared__ uint32_t lh[];
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) atomicAdd(&lh[length_bin(offsets, s, nbins)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x)
        if (lh[i]) atomicAdd(&hist[i], lh[i]);
}

// Exclusive scan of hist[nbins] into cursor[nbins], hist zeroed (one block; nbins <= 4 * kOrderThreads).
__global__ __launch_bounds__(kOrderThreads) void order_scan_kernel(uint32_t* __restrict__ hist,
                                                                   uint32_t* __restrict__ cursor, uint32_t nbins) {
    __shared__ uint32_t part[kOrderThreads];
    const uint32_t t = threadIdx.x;
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        v[q] = i < nbins ? hist[i] : 0u;
        if (i < nbins) hist[i] = 0u;
        sum += v[q];
    }
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < kOrderThreads; d <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t x = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        if (i < nbins) cursor[i] = run;
        run += v[q];
    }
}

__global__ __launch_bounds__(kOrderThreads) void order_place_kernel(const uint64_t* __restrict__ offsets, uint64_t n,
                                                                    uint64_t chunk, uint32_t* __restrict__ cursor,
                                                                    uint32_t nbins, uint32_t* __restrict__ order) {
    extern __shared__ uint32_t lh[];  // [0, nbins): block counts, then block cursors
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) atomicAdd(&lh[length_bin(offsets, s, nbins)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x)
        if (lh[i]) lh[i] = atomicAdd(&cursor[i], lh[i]);  // reserve this block's range of bin i
    __syncthreads();
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) {
        const uint32_t slot = atomicAdd(&lh[length_bin(offsets, s, nbins)], 1u);
        order[slot] = static_cast<uint32_t>(s);
    }
}

// ------------------------------------------------------------------------------------------------
// MSV filter P-values (msv.h): one thread per sequence, HBM-bound elementwise
// (12 B read + 8 B written per sequence).  Same float/double steps as msv_stats.cpp's host path.
// ------------------------------------------------------------------------------------------------
__device__ __host__ inline double msv_pvalue_of(float score, uint64_t L, float mu, float lambda) {
    if (L == 0) return 1.0;  // empty sequence: score -inf, and L log(p1) would be 0 * -inf
    const float p1 = static_cast<float>(L) / static_cast<float>(L + 1);
    const float nullsc = static_cast<float>(static_cast<double>(L) * log(static_cast<double>(p1)) +
                                            log(1.0 - static_cast<double>(p1)));
    const float bits = (score - nullsc) / 0.69314718055994529f;
    const double y = static_cast<double>(lambda) * (static_cast<double>(bits) - static_cast<double>(mu));
    const double ey = -exp(-y);
    return fabs(ey) < 5e-9 ? -ey : 1.0 - exp(ey);
}

__global__ __launch_bounds__(256) void msv_pvalues_kernel(const float* __restrict__ scores,
                                                          const uint64_t* __restrict__ offsets, uint64_t n, float mu,
                                                          float lambda, double* __restrict__ out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) out[i] = msv_pvalue_of(scores[i], offsets[i + 1] - offsets[i], mu, lambda);
}

hipError_t launch_pvalues(const float* scores, const uint64_t* offsets, uint64_t n, float mu, float lambda,
                          double* pvalues, hipStream_t stream) {
    const uint64_t blocks = (n + 255) / 256;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(msv_pvalues_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream, scores, offsets,
                       n, mu, lambda, pvalues);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Variant table: every compiled (G, S, WAVES) instantiation.  The host picks the one whose G*S
// covers LENG with the least estimated cost (the analog of the reference's should_specialize,
// which bakes sizes into the OpenCL program with -D defines, MSV_HMM.cpp:322-337).
// ------------------------------------------------------------------------------------------------
#define MSV_VARIANT(G_, S_, W_, P_, D_)                                                                   \
    Variant{G_, S_, W_, P_, D_, lds_rows_for(G_, S_), lds_rows_for(G_, S_) < kTableRows,                  \
            reinterpret_cast<const void*>(                                                                 \
                &msv_batch_kernel<G_, S_, W_, P_, (lds_rows_for(G_, S_) < kTableRows), D_>),               \
            "msv_g" #G_ "_s" #S_ "_w" #W_ "_p" #P_ "_d" #D_}

// Split layout (G = 32 or 64): SA states per lane from LDS (20 rows), S - SA from L2.
#define MSV_SPLIT_VARIANT(G_, S_, SA_, W_, P_)                                                            \
    Variant{G_, S_, W_, P_, 1, kAminoAcids, false,                                                        \
            reinterpret_cast<const void*>(&msv_batch_kernel<G_, S_, W_, P_, false, 1, SA_>),               \
            "msv_g" #G_ "_s" #S_ "_a" #SA_ "_w" #W_ "_p" #P_ "_d1", SA_}

static const Variant kVariants[] = {
#include "msv_variants.inc"
};

const Variant* variants(int* count) {
    *count = static_cast<int>(sizeof(kVariants) / sizeof(kVariants[0]));
    return kVariants;
}

hipError_t launch_variant(const Variant& v, dim3 grid, const KernelArgs& args, hipStream_t stream, hipEvent_t start,
                          hipEvent_t stop) {
    void* params[] = {const_cast<KernelArgs*>(&args)};
    if (start || stop) return hipExtLaunchKernel(v.fn, grid, dim3(v.waves * 64), params, 0, stream, start, stop, 0);
    return hipLaunchKernel(v.fn, grid, dim3(v.waves * 64), params, 0, stream);
}

// Small batches (n <= kSmallOrderPer * kOrderThreads): the whole counting sort in ONE launch and one
// workgroup (histogram, scan and cursors in LDS, no memset), lengths held in registers between the
// passes.  Replaces 4 dependent launches (~17 us of launch latency) by one (~5 us).
constexpr int kSmallOrderPer = 16;

__global__ __launch_bounds__(kOrderThreads) void order_small_kernel(const uint64_t* __restrict__ offsets, uint32_t n,
                                                                    uint32_t nbins, uint32_t* __restrict__ order) {
    extern __shared__ uint32_t lh[];  // [nbins] counts -> cursors, [kOrderThreads] scan partials
    uint32_t* part = lh + nbins;
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < nbins; i += kOrderThreads) lh[i] = 0;
    uint32_t bin[kSmallOrderPer];
#pragma unroll
    for (int k = 0; k < kSmallOrderPer; ++k) {
        const uint32_t s = t + k * kOrderThreads;
        bin[k] = s < n ? length_bin(offsets, s, nbins) : 0xFFFFFFFFu;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmallOrderPer; ++k)
        if (bin[k] != 0xFFFFFFFFu) atomicAdd(&lh[bin[k]], 1u);
    __syncthreads();
    // exclusive scan of lh[0..nbins): 4 consecutive bins per thread, Hillis-Steele over threads
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        v[q] = i < nbins ? lh[i] : 0u;
        sum += v[q];
    }
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < kOrderThreads; d <<= 1) {
        const uint32_t x = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        if (i < nbins) lh[i] = run;
        run += v[q];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmallOrderPer; ++k)
        if (bin[k] != 0xFFFFFFFFu) order[atomicAdd(&lh[bin[k]], 1u)] = t + k * kOrderThreads;
}

hipError_t launch_order(const uint64_t* offsets, uint64_t n, uint32_t* scratch_hist, uint32_t nbins, uint32_t* order,
                        hipStream_t stream) {
    if (nbins > 4 * kOrderThreads) return hipErrorInvalidValue;
    if (n <= static_cast<uint64_t>(kSmallOrderPer) * kOrderThreads) {
        const size_t lds = (nbins + kOrderThreads) * sizeof(uint32_t);
        hipLaunchKernelGGL(order_small_kernel, dim3(1), dim3(kOrderThreads), lds, stream, offsets,
                           static_cast<uint32_t>(n), nbins, order);
        return hipGetLastError();
    }
    const uint64_t blocks = std::min<uint64_t>(256, (n + 511) / 512);
    const uint64_t chunk = (n + blocks - 1) / blocks;
    const size_t lds = nbins * sizeof(uint32_t);
    hipLaunchKernelGGL(order_count_kernel, dim3(blocks), dim3(kOrderThreads), lds, stream, offsets, n, chunk,
                       scratch_hist, nbins);
    hipLaunchKernelGGL(order_scan_kernel, dim3(1), dim3(kOrderThreads), 0, stream, scratch_hist,
                       scratch_hist + nbins, nbins);
    hipLaunchKernelGGL(order_place_kernel, dim3(blocks), dim3(kOrderThreads), lds, stream, offsets, n, chunk,
                       scratch_hist + nbins, nbins, order);
    return hipGetLastError();
}

}  // namespace msvk
