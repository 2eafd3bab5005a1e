// k_rowown.hpp -- the row-owner split-GEMM machinery shared by the fp32 tower kernels of k_head_s3.hip
// (tower layer 1, gathered) and k_tail_s3.hip (layers 2 + 3 + head), gfx950.
//
// A block of 8 waves (two per SIMD) owns 128 rows; a wave owns 16 rows and ALL 416 columns of a layer.
// The MFMA runs with the operands swapped (D = W x^T, v_mfma_f32_16x16x32_bf16 with the weight plane as
// A), so lane (r16, g) holds outputs n = 16 t + 4 g .. + 3 of its sample r16 -- the K values that lane
// group g feeds the next layer at the split engine's positions (k_gemm.hpp kPrecS3: step c, half h,
// K = 32 c + 16 h + 4 g + q).  The weights (fp32 pre-split into three bf16 planes, W3 [steps][3][416][32])
// stream through LDS in "units" of one K step x one column half (13 tiles x 3 planes x 1 KiB = 39 KiB), a
// 3-slot ring: unit U + 2's DMAs are issued during unit U, one per column tile, one barrier per unit.
#pragma once

#include "k_gemm.hpp"

namespace rmx {
namespace rowown {

constexpr int kQBM = 128;                    // rows per row block
constexpr int kQW = 8;                       // waves
constexpr int kQThreads = kQW * 64;
constexpr int kQNT = 25;                     // computed column tiles (N = 400)
constexpr int kQN = 416;                     // Npad: packed rows of W per plane and K step
constexpr int kQUT = 13;                     // column tiles per unit (one half of Npad)
constexpr int kQUnit = 3 * kQUT * 16 * 64;   // bytes per unit: 3 planes x 208 rows x 64 B = 39,936
constexpr int kQIns = kQUnit / 1024;         // 1-KiB DMA instructions per unit (39)
constexpr int kQQ = (kQIns + kQW - 1) / kQW; // per wave (5; wave 7's fifth repeats instruction 38)
constexpr int kQSlots = 3;
static_assert(kQQ == 5 && kQIns == 39, "the static vmcnt counts assume 5 weight DMAs per wave per unit");

// Diagnostic builds only (timing probes, wrong results; never set in librmx.so): 1 = no DMAs after the
// prologue, 2 = no MFMAs
#ifndef RMX_QTAIL_DIAG
#define RMX_QTAIL_DIAG 0
#endif
// the tiles of a unit that carry its five weight DMAs (timing A/B)
#ifndef RMX_QTAIL_DOFF
#define RMX_QTAIL_DOFF 0
#endif
#ifndef RMX_QTAIL_DSTRIDE
#define RMX_QTAIL_DSTRIDE 1
#endif


// this wave's DMA q of a unit whose planes start at `src` into the slot at `dst` (LDS byte offset).
// Instruction ins = w + 8 q fills unit rows [16 ins, 16 ins + 16): plane ins / 13, tile ins % 13; lane L
// writes physical 16-B slot L & 3 of row L >> 2, so it loads logical slot swz_slot(row, L & 3) (the
// swizzle is an involution; the key of row 16 t + (L >> 2) depends on L only): lo = its element offset.
// (PS: rows of W per plane and K step -- 416 for the tower layers, 208 for the CIN's)
template <int PS = kQN>
__device__ __forceinline__ void q_dma(const bf16_t* src, char* lds, int slot, int w, int q, int lo) {
  int ins = w + q * kQW;
  ins = ins < kQIns ? ins : kQIns - 1;
  const int pl = ins / kQUT, t = ins - pl * kQUT;
  int l = lo;
  asm volatile("" : "+v"(l));  // formed here: hoisted, the 130 per-unit sources of layer 3 spilled
  const bf16_t* s = src + (pl * PS + t * 16) * 32 + l;
  lds_dma<16>(s, lds + slot * kQUnit + ins * 1024);
}

__device__ __forceinline__ int q_next(int s) { return s == kQSlots - 1 ? 0 : s + 1; }

// per-lane byte offset of the weight fragments (row r16 of a tile, logical slot g), opaque so the
// fragment addresses are formed per use
__device__ __forceinline__ int q_fbase(int lane) {
  int fb = (lane & 15) * 64 + swz_slot(lane & 15, lane >> 4) * 16;
  asm volatile("" : "+v"(fb));
  return fb;
}

// no extra vector-memory instructions in a unit (q_unit's default)
struct QNoExtra {
  __device__ __forceinline__ void operator()(int) const {}
};

// One unit: NT column tiles (local tiles 0 .. NT - 1 of the unit's half) of one K step.  acc[T0 + t] +=
// W_t h^T on the split planes (ah, am, al) of this wave's 16 rows; dma(q) issues the wave's q-th DMA of
// unit U + 2, one per tile.  The fragments of tile t + 2 are read while tile t's MFMAs run.  extra(t) may
// issue more vector-memory instructions at tile t (after that tile's plane DMA): a caller's own DMAs spread
// over the MFMA stream instead of issued ahead of it.
// DOFF: the tile that carries the unit's first weight DMA (the rest follow one per tile); kernels whose two
// waves per SIMD issue their DMAs at different tiles pass it per wave half (k_fused_s3.hip)
template <int NT, int T0, int NA, int PF = 2, int PS = kQN, int DOFF = RMX_QTAIL_DOFF, class X = QNoExtra>
__device__ __forceinline__ void q_unit(const char* ub, int fb, const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                       f32x4 (&acc)[NA], const bf16_t* dsrc, char* lds, int dslot, int w, int lo,
                                       bool mm = true, const X& extra = X()) {
  f32x4 bq[PF + 1][3];
  int fbu = fb;
  asm volatile("" : "+v"(fbu));
  auto ldb = [&](int t, f32x4* b) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) b[pl] = *reinterpret_cast<const f32x4*>(ub + fbu + pl * (kQUT * 1024) + t * 1024);
  };
#pragma unroll
  for (int t = 0; t < PF; ++t) ldb(t, bq[t]);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t + PF < NT) ldb(t + PF, bq[(t + PF) % (PF + 1)]);
    // DMA q rides tile DOFF + q * RMX_QTAIL_DSTRIDE
    constexpr int kD0 = DOFF, kDS = RMX_QTAIL_DSTRIDE;
    static_assert(kD0 + (kQQ - 1) * kDS < kQUT - 1, "every unit (12 or 13 tiles) carries all its DMAs");
    if (t >= kD0 && (t - kD0) % kDS == 0 && (t - kD0) / kDS < kQQ && !(RMX_QTAIL_DIAG & 1))
      q_dma<PS>(dsrc, lds, dslot, w, (t - kD0) / kDS, lo);
    extra(t);
    __builtin_amdgcn_sched_barrier(0);
    const f32x4* b = bq[t % (PF + 1)];
    const bf16x8 bh = __builtin_bit_cast(bf16x8, b[0]);
    const bf16x8 bm = __builtin_bit_cast(bf16x8, b[1]);
    const bf16x8 bl = __builtin_bit_cast(bf16x8, b[2]);
    if constexpr (RMX_QTAIL_DIAG & 2) {
      acc[T0 + t] += b[0] + b[1] + b[2] + __builtin_bit_cast(f32x4, ah);
      continue;
    }
    if (!mm) continue;  // a wave without rows this row block (QRows half blocks): DMAs only
    f32x4 d = acc[T0 + t];
    // the engine's product order (k_gemm.hpp compute_step_s3), operands swapped: smallest terms first
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, am, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, am, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, ah, d, 0, 0, 0);
    acc[T0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, d, 0, 0, 0);
  }
}

// the DMAs of q_unit without its MFMAs: a wave that owns no rows this row block (a half block's waves
// 4 .. 7) keeps the ring and the static vmcnt counts
template <int PS = kQN>
__device__ __forceinline__ void q_dma_only(const bf16_t* dsrc, char* lds, int dslot, int w, int lo) {
#pragma unroll
  for (int q = 0; q < kQQ; ++q) q_dma<PS>(dsrc, lds, dslot, w, q, lo);
}

// Row blocks of a persistent row-owner launch (grid G): full 128-row blocks, round-robin.  When the last
// round would leave at least half the CUs idle, its rows go out as 64-row half blocks instead: waves 0 .. 3
// own the rows, waves 4 .. 7 keep the weight ring and the barriers but run no MFMAs, so the round costs
// about half a round (B = 49,152 on 256 CUs: 1.5 rounds instead of 2; B = 16,384: half a round, not one).
struct QRows {
  int M, G, nfull, nhalf;  // nfull full blocks, then nhalf half blocks from row nfull * 128
  __device__ __forceinline__ int nf(int b) const { return b < nfull ? (nfull - 1 - b) / G + 1 : 0; }
  __device__ __forceinline__ int nit(int b) const { return nf(b) + (b < nhalf ? 1 : 0); }
  // iteration it of block b: first row and the number of waves that own rows (0: none -- past the end)
  __device__ __forceinline__ void desc(int b, int it, int& row0, int& nw) const {
    const int n = nf(b);
    if (it < n) {
      row0 = (b + it * G) * kQBM;
      nw = kQW;
    } else if (it == n && b < nhalf) {
      row0 = nfull * kQBM + b * (kQBM / 2);
      nw = kQW / 2;
    } else {
      row0 = M;
      nw = 0;
    }
  }
};

// host: the row blocks of M rows on ncu CUs and the grid that runs them (knob "half_blocks", default 1 since
// measured: DeepFM B = 49,152 137-161 -> 180-182 M examples/s, profiles/r04/ab_round4_first.txt)
inline QRows q_rows(int M, int ncu, int& grid) {
  QRows r{M, 1, 0, 0};
  const int nb = (M + kQBM - 1) / kQBM;
  ncu = ncu > 0 ? ncu : 1;
  const int R = (nb + ncu - 1) / ncu, last = nb - (R - 1) * ncu;
  if (tuning_get("half_blocks", 1) != 0 && 2 * last <= ncu) {
    r.nfull = (R - 1) * ncu;
    r.nhalf = (M - r.nfull * kQBM + kQBM / 2 - 1) / (kQBM / 2);
    grid = r.nfull > 0 ? ncu : (r.nhalf < ncu ? r.nhalf : ncu);
  } else {
    r.nfull = nb;
    grid = nb < ncu ? nb : ncu;
  }
  r.G = grid;
  return r;
}

// host: whether the launch's (half) row blocks occupy every CU at least once
inline bool q_fills(int M, int ncu) {
  int grid = 0;
  (void)q_rows(M, ncu, grid);
  return grid >= ncu;
}

// unit start: this unit's DMAs (issued two units ago) have landed for this wave (N = vector-memory
// instructions the wave issued during the previous unit), then for every wave; the slot the next DMAs
// overwrite was read by every wave before this barrier
template <int N>
__device__ __forceinline__ void q_enter() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// the ReLU mask bits of a lane's outputs (training, k_layer_s3.hip): tile t's four outputs (n = 16 t + 4 g + q)
// at bits 4 t + q of the lane's 4-word group (100 of 128 bits for 25 tiles).  v is a ReLU output (> 0 or +0),
// so its bit is min(bits(v), 1): integer ops only (compares would hold 100 lane masks in SGPR pairs: the
// head spilled 179 SGPRs with them)
__device__ __forceinline__ void bits_set(uint32_t (&mb)[4], int t, const f32x4& v) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = 4 * t + q;
    mb[i >> 5] |= min(__float_as_uint(v[q]), 1u) << (i & 31);
  }
}

__device__ __forceinline__ f32x4 relu4(f32x4 v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
  return v;
}

}  // namespace rowown
}  // namespace rmx
