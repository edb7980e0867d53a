// msv_coop.hip -- the cooperative plan: ONE sequence per workgroup, its DP row spread over the W waves
// of the workgroup (one per SIMD of a CU), for batches of fewer sequences than the chip has CUs -- the
// shape of the reference's own benchmark programs, which score one sequence per call
// (algorithms/benchmark_helper.hpp:19-38, benchmark_MSV_1400.cpp:8-13: 1400.hmm x 3 x 3500 residues).
//
// With one sequence per wave (the latency plan) a 1400-state row is ~100 VALU issued by ONE wave,
// latency-bound at ~0.24 us per row.  Here each of the W waves owns a contiguous quarter of the row
// (64 lanes x S states) and issues ~1/W of the instructions.  The only cross-wave dependencies of a
// row t are (MSV_HMM.cpp:100-111):
//   * the j-1 neighbour of a wave's first state (the previous wave's last state at row t-1), and
//   * B(t-1) = max(N, J) + move, J being the max over ALL states.
// Neither is exchanged per row:
//   * HALO: wave w's lanes also cover the K >= 16 states just below its own (the last K states of wave
//     w-1, recomputed redundantly).  At the start of a 16-row block the halo lanes are loaded with
//     wave w-1's exact values; the halo's first state has no left neighbour (-inf), so after r rows of
//     the block only its first r+1 states can be wrong -- and wrong values are LOWER bounds (a max with
//     -inf instead of the true neighbour), which leave every max (E, J) exact.  With K >= 16 the wave's
//     own states stay exact for the whole block.
//   * SPECULATION: B = N + move, exact while every J partial stays below N (the common case off
//     homologous segments); every row ORs (J >= N) into a flag.  At the block's end the W waves
//     exchange flags and halos with ONE barrier; a flagged block is rolled back to its saved start and
//     re-run with the exact per-row B (a barrier per row to max the waves' J).
// The last partial block of a sequence (L mod 16 rows) runs that exact way too.  Bit-exact for every
// input: the same IEEE ops in the same order per state as the batch kernel (msv_kernel_body.inc).
#include "msv_kernel_impl.h"

namespace msvk {

template <int W, int S>
__global__ __launch_bounds__(W * 64) void msv_coop_kernel(const KernelArgs a) {
    static_assert(S % 2 == 0 && S >= 2 && S <= 8, "float2 chunks");
    static_assert(W % 4 == 0 || W == 2, "waves per workgroup");
    constexpr int HL = (16 + S - 1) / S;  // halo lanes per wave (K = HL * S >= 16 states)
    constexpr int H = S / 2;              // float2 chunks per lane
    constexpr int ROW2 = W * H * 64;      // float2 per residue row of the table
    constexpr int BLKN = 16;
    __shared__ float2 tab[kTableRows * ROW2];
    __shared__ float halo[2][W][HL * S];
    __shared__ uint32_t flag[2][W];
    __shared__ float jx[2][W];

    const float2* et = reinterpret_cast<const float2*>(a.etab);
    for (int i = threadIdx.x; i < kTableRows * ROW2; i += W * 64) tab[i] = et[i];
    __syncthreads();

    const float NINF = -__builtin_inff();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t blk_lane = static_cast<uint32_t>(lane & (BLKN - 1));
    const float trBMk = a.tr_B_Mk, tEJ = a.tr_E_J;
    const uint8_t* __restrict__ res = a.residues;
    // this lane's chunks of residue row r: tab[r * ROW2 + (w * H + h) * 64 + lane]
    const uint32_t lane_off = static_cast<uint32_t>((w * H * 64 + lane) * 8);
    auto row_ptr = [&](uint32_t r) -> const float2* {
        uint32_t off;
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(off) : "v"(r), "s"(static_cast<uint32_t>(ROW2 * 8)), "v"(lane_off));
        return reinterpret_cast<const float2*>(reinterpret_cast<const char*>(tab) + off);
    };
    struct Ring {
        float2 v[H];
    };
    auto fill = [&](Ring& rg, const float2* p) {
#pragma unroll
        for (int h = 0; h < H; ++h) rg.v[h] = p[h * 64];
    };

    int par = 0;   // halo / flag buffer of this block
    int rpar = 0;  // J exchange buffer of this exact row
    for (uint64_t idx = blockIdx.x; idx < a.n; idx += gridDim.x) {
        const uint32_t s = a.order ? a.order[idx] : static_cast<uint32_t>(idx);
        if (s >= a.n) {  // an order entry outside the batch (msv_kernel_body.inc begin)
            if (threadIdx.x == 0) {
                a.scores[idx] = __uint_as_float(0x7fc00000u);
                atomicOr(a.errors, kErrBadOrder);
            }
            continue;
        }
        const uint64_t o0 = a.offsets[s], o1 = a.offsets[s + 1];
        const uint64_t L = o1 - o0;
        if (L == 0 || L >= a.lentab_n) {  // C_0 = -inf (MSV_HMM.cpp:86,112); too long: NaN + error
            if (threadIdx.x == 0) {
                a.scores[s] = L == 0 ? NINF : __uint_as_float(0x7fc00000u);
                if (L != 0) atomicOr(a.errors, kErrTooLong);
            }
            continue;
        }
        const float2 lm = a.lentab[L];
        const float loop = lm.x, move = lm.y;
        const uint32_t last = static_cast<uint32_t>(L - 1);
        const uint8_t* sr = res + o0;

        float M[S];
#pragma unroll
        for (int k = 0; k < S; ++k) M[k] = NINF;
        float J = NINF, N = 0.f, B = move, nbr = NINF;  // row 0 (MSV_HMM.cpp:86,96-97)
        uint32_t pos = 0;
        uint8_t nxt = sr[min(blk_lane, last)];
        uint32_t cur = 0;
        Ring ra, rb;  // emission chunks of the even / odd rows, requested two rows ahead

        auto cells = [&](Ring& rg) __attribute__((always_inline)) {
            const float Bt = B + trBMk;
            nbr = shift_in<64>(M[S - 1], nbr);
#pragma unroll
            for (int h = H - 1; h >= 0; --h) {  // highest states first: M[k-1] is still the previous row's
                const float2 ev = rg.v[h];
                M[2 * h + 1] = ev.y + fmaxf(M[2 * h], Bt);
                M[2 * h] = ev.x + fmaxf(h == 0 ? nbr : M[2 * h > 0 ? 2 * h - 1 : 0], Bt);
            }
        };
        auto lane_E = [&]() {
            float e = M[0];
#pragma unroll
            for (int k = 1; k < S; ++k) e = fmaxf(e, M[k]);
            return e;
        };
        // The exact row (MSV_HMM.cpp:100-111): B from the max of every wave's J (one barrier).
        auto exact_row = [&](uint32_t code) __attribute__((always_inline)) {
            Ring rg;
            fill(rg, row_ptr(code));
            cells(rg);
            J = fmaxf(J + loop, lane_E() + tEJ);
            N = N + loop;
            const float jw = group_max<64>(J);
            if (lane == 0) jx[rpar][w] = jw;
            __syncthreads();
            float jg = jx[rpar][0];
#pragma unroll
            for (int q = 1; q < W; ++q) jg = fmaxf(jg, jx[rpar][q]);
            rpar ^= 1;
            B = fmaxf(N, jg) + move;
            ++pos;
        };
        // End of a block: publish the last HL lanes' states (the next wave's halo) and this wave's flag.
        auto publish = [&](bool viol) __attribute__((always_inline)) {
            if (lane >= 64 - HL) {
#pragma unroll
                for (int k = 0; k < S; ++k) halo[par][w][(lane - (64 - HL)) * S + k] = M[k];
            }
            const bool any = __any(viol);
            if (lane == 0) flag[par][w] = any ? 1u : 0u;
        };
        auto refresh_halo = [&]() __attribute__((always_inline)) {
            if (w > 0 && lane < HL) {
#pragma unroll
                for (int k = 0; k < S; ++k) M[k] = halo[par][w - 1][lane * S + k];
            }
        };

        while (pos + BLKN <= L) {
            cur = min(static_cast<uint32_t>(nxt), static_cast<uint32_t>(kPoisonRow));
            nxt = sr[min(pos + BLKN + blk_lane, last)];
            float save_M[S];
#pragma unroll
            for (int k = 0; k < S; ++k) save_M[k] = M[k];
            const float save_J = J, save_N = N, save_B = B, save_nbr = nbr;
            bool viol = false;
            fill(ra, row_ptr(row_bcast_lane<0>(cur)));
            fill(rb, row_ptr(row_bcast_lane<1>(cur)));
            // Rows software-pipelined across scheduling regions: the tail of row P (E, J, N, flag, B)
            // with the cells of row P+1, which need only row P's cells and B = N + move.
            auto tail = [&]() __attribute__((always_inline)) {
                J = fmaxf(J + loop, lane_E() + tEJ);
                N = N + loop;
                viol |= J >= N;
                B = N + move;  // == max(N, J) + move while no J partial reaches N
            };
            [&]<int... P>(std::integer_sequence<int, P...>) {
                ((
                     [&] {
                         if constexpr (P > 0) tail();
                         Ring& rg = (P & 1) ? rb : ra;
                         cells(rg);
                         if constexpr (P + 2 < BLKN) fill(rg, row_ptr(row_bcast_lane<(P + 2 < BLKN ? P + 2 : 0)>(cur)));
                         __builtin_amdgcn_sched_barrier(0);
                     }()),
                 ...);
            }(std::make_integer_sequence<int, BLKN>{});
            tail();
            pos += BLKN;
            publish(viol);
            __syncthreads();
            bool any = false;
#pragma unroll
            for (int q = 0; q < W; ++q) any |= flag[par][q] != 0;
            if (__builtin_expect(any, 0)) {
                // some row needed the waves' J for B: redo the block exactly from its saved start
#pragma unroll
                for (int k = 0; k < S; ++k) M[k] = save_M[k];
                J = save_J;
                N = save_N;
                B = save_B;
                nbr = save_nbr;
                pos -= BLKN;
                [&]<int... P>(std::integer_sequence<int, P...>) {
                    (exact_row(row_bcast_lane<P>(cur)), ...);
                }(std::make_integer_sequence<int, BLKN>{});
                publish(false);
                __syncthreads();
            }
            refresh_halo();
            par ^= 1;
        }
        // the last L mod 16 rows, exactly
        const uint32_t rem = static_cast<uint32_t>(L) - pos;  // uniform
        if (rem > 0) {
            cur = min(static_cast<uint32_t>(nxt), static_cast<uint32_t>(kPoisonRow));
            [&]<int... P>(std::integer_sequence<int, P...>) {
                ((P < static_cast<int>(rem) ? exact_row(row_bcast_lane<P>(cur)) : void()), ...);
            }(std::make_integer_sequence<int, BLKN>{});
        }
        // score = C_L + move, C == J (tr_E_C == tr_E_J; msv_device.cpp installs this plan only then)
        const float jw = group_max<64>(J);
        if (lane == 0) jx[rpar][w] = jw;
        __syncthreads();
        if (threadIdx.x == 0) {
            float C = jx[rpar][0];
#pragma unroll
            for (int q = 1; q < W; ++q) C = fmaxf(C, jx[rpar][q]);
            const float sc = C + move;
            a.scores[s] = sc;
            if (!(sc <= 3.402823466e38f)) atomicOr(a.errors, kErrBadResidue);  // poison row hit
        }
        rpar ^= 1;
        __syncthreads();  // the LDS exchange buffers are reused by the next sequence
    }
}

#define MSV_COOP_VARIANT(W_, S_)                                                                            \
    CoopVariant{W_, S_, (16 + S_ - 1) / S_ * S_, reinterpret_cast<const void*>(&msv_coop_kernel<W_, S_>), \
                "msv_coop_w" #W_ "_s" #S_}

static const CoopVariant kCoop[] = {MSV_COOP_VARIANT(4, 2), MSV_COOP_VARIANT(4, 4), MSV_COOP_VARIANT(4, 6)};

const CoopVariant* coop_variants(int* count) {
    *count = static_cast<int>(sizeof(kCoop) / sizeof(kCoop[0]));
    return kCoop;
}

}  // namespace msvk
