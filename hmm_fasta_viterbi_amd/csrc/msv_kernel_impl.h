// msv_kernel_impl.h -- the MSV kernel templates (msv_batch_kernel, msv_grid_kernel) and the variant-table
// macros, shared by the translation units that instantiate the variant family (msv_kernel_part.hip,
// compiled once per msv_variants_<k>.inc so the family builds in parallel).  See msv_kernel.hip for
// the mapping of the recurrence onto CDNA4.
#pragma once
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
constexpr int DPP_WAVE_SHR1 = 0x138;   // wave_shr:1 (the whole wave, one lane down)

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
        return dpp<DPP_WAVE_SHR1>(old, last);  // one move; lane 0 has no source and keeps `old`
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

// WIDE blocks (zero-copy twins of BLK variants, one stream per lane group): the current and next 64-row
// superblocks (one dword per lane), the next superblock's address and the load clamp, the index of the
// next block, the next block (taken from the current superblock by ds_bpermute).  Kept out of Stream:
// any new Stream field moved the register assignment of every other variant.
struct WideBlocks {
    uint32_t wcur, wnext, nsh, snext, e3, wr, nxw;  // (nsh: wnext's pending shift, see load_w)
};
struct NoWideBlocks {};

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
// RPFO > 0 overrides the rows of residue prefetch (the zero-copy twins below).
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0, int RPFO = 0>
__global__ __launch_bounds__(WAVES * 64) void msv_batch_kernel(const KernelArgs a) {
#define MSV_BLOCK blockIdx.x
#define MSV_BLOCKS gridDim.x
#include "msv_kernel_body.inc"
#undef MSV_BLOCK
#undef MSV_BLOCKS
}

// Several profiles' batches in ONE launch (msv_score_grid of a few sequences: each profile's own
// launch would last one sequence's rows, and separate launches serialise on the process's few hardware
// queues).  Workgroups [p * per_profile, (p + 1) * per_profile) score profile p with g.p[p] -- its
// table in this variant's layout, its counter slot, scores and specials -- exactly as msv_batch_kernel
// would with a grid of per_profile workgroups.  The arguments travel in the kernarg segment (copied
// at launch: nothing for the host to keep alive).
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0, int RPFO = 0>
__global__ __launch_bounds__(WAVES * 64) void msv_grid_kernel(const GridArgs g) {
    const uint32_t profile = blockIdx.x / g.per_profile;
    const uint32_t per_profile = g.per_profile;
    const uint32_t block_in_profile = blockIdx.x - profile * per_profile;
    const KernelArgs a = g.p[profile];
#define MSV_BLOCK block_in_profile
#define MSV_BLOCKS per_profile
#include "msv_kernel_body.inc"
#undef MSV_BLOCK
#undef MSV_BLOCKS
}

// The grid kernel exists for the one-sequence-per-wave (G = 64) variants only: the plans that a few
// sequences take.
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0>
constexpr const void* grid_fn() {
    if constexpr (G == 64 && D == 1) return reinterpret_cast<const void*>(&msv_grid_kernel<G, S, WAVES, PF, BIG, D, SA>);
    else return nullptr;
}

// Zero-copy twins: the same variant reading its residues two rows ahead -- which for 16/32-lane rows
// means residue BLOCKS (one byte load per lane per 16 rows, a block ahead) -- for launches whose
// residues sit in page-locked host memory.  A row of 41-96 states is long enough that one row of
// prefetch hides an HBM/L2 load, not a PCIe round trip at each 128-B line: cfg3 read in place 2.945 vs
// 2.856 ms with the twin, while from HBM it is 0.3-0.7% slower on 1400/1901.hmm (2% faster on
// 1001.hmm) -- profiles/r02_zero_copy_twins.jsonl.  Split variants already prefetch two rows.
// Rows of up to 40 states already read residue blocks (one 16-byte request per group per 16 rows):
// the twins of those with two-rows-ahead emission rings (PF <= 2) read WIDE blocks, 64-byte requests
// (msv_kernel_body.inc): cfg2's call 0.228 -> 0.223 ms, 200.hmm x 2000 (64-lane plan) 0.126 -> 0.121 ms;
// the whole-row-ring variants (PF = S/4 > 2) were slower with them (400.hmm x 20k 0.415 -> 0.46 ms) and
// keep their 16-byte blocks -- profiles/r03_ab_zero_copy_wide.jsonl.
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0>
constexpr const void* zc_fn() {
    if constexpr ((G == 16 || G == 32) && D == 1 && !BIG && SA == 0 && S > 40)
        return reinterpret_cast<const void*>(&msv_batch_kernel<G, S, WAVES, PF, BIG, D, SA, 2>);
    else if constexpr (G >= 16 && D == 1 && !BIG && SA == 0 && residue_prefetch<S>() > 1 && PF <= 2)
        return reinterpret_cast<const void*>(&msv_batch_kernel<G, S, WAVES, PF, BIG, D, SA, kWideBlocks>);
    else return nullptr;
}

// CLOCK twins (RPFO = kClockTwin): the plans bench.py's configs run -- 16 x 8 (cfg2), 16 x 88 (cfg3, cfg4),
// the 32 x 76 split (cfg5) -- with stamps that also record s_memtime, for roofline.clock_GHz.  A separate
// instantiation: adding the ticks to the production kernels renamed their registers and cost cfg2 1.3%
// (profiles/r04_ab_stamp_clock.jsonl).
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0>
constexpr const void* clock_fn() {
    if constexpr (D == 1 && !BIG && PF == 2 &&
                  ((G == 16 && (S == 8 || S == 88) && SA == 0) || (G == 32 && S == 76 && SA == 64)))
        return reinterpret_cast<const void*>(&msv_batch_kernel<G, S, WAVES, PF, BIG, D, SA, kClockTwin>);
    else return nullptr;
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
            "msv_g" #G_ "_s" #S_ "_w" #W_ "_p" #P_ "_d" #D_, 0,                                              \
            grid_fn<G_, S_, W_, P_, (lds_rows_for(G_, S_) < kTableRows), D_>(),                            \
            zc_fn<G_, S_, W_, P_, (lds_rows_for(G_, S_) < kTableRows), D_>(),                              \
            clock_fn<G_, S_, W_, P_, (lds_rows_for(G_, S_) < kTableRows), D_>()}

// Split layout (G = 32 or 64): SA states per lane from LDS (20 rows), S - SA from L2.
#define MSV_SPLIT_VARIANT(G_, S_, SA_, W_, P_)                                                            \
    Variant{G_, S_, W_, P_, 1, kAminoAcids, false,                                                        \
            reinterpret_cast<const void*>(&msv_batch_kernel<G_, S_, W_, P_, false, 1, SA_>),               \
            "msv_g" #G_ "_s" #S_ "_a" #SA_ "_w" #W_ "_p" #P_ "_d1", SA_, grid_fn<G_, S_, W_, P_, false, 1, SA_>(),  \
            nullptr, clock_fn<G_, S_, W_, P_, false, 1, SA_>()}

}  // namespace msvk
