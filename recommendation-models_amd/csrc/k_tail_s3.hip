// k_tail_s3.hip -- the fp32 tower tail in one persistent kernel on the split GEMM (gfx950): DeepFM / DNN /
// xDeepFM / DCN / PNN fp32 towers, BASELINE.json configs[1] and [2].
//
// The last hidden Linear + ReLU and the output Linear + head of an fp32 tower
// (model/encoder/HigherOrderEncoder.scala:34-59: Linear(400 -> 400) + ReLU, then the last
// Linear(400 -> 400) + ReLU whose output feeds Linear(400 -> 1); the heads of DeepFM.scala:54-80 and
// the other models: CAddTable + Sigmoid):
//   h2 = ReLU(h1 W2^T + b2)                         kept in the wave's registers, never written to HBM
//   y  = sum_n ReLU(h2 W3^T + b3)[n] wo[n] (+ bo);  p = sigmoid(pre + (pre2 | rowsum + y) + beta)
// Why: as two split-GEMM launches, layer 2 writes h2 (105 MB at B = 65,536) in one burst at the end of
// each round of blocks and layer 3 reads it back; the timing-only builds of round 3 put the
// stored-activation epilogue at ~15 % of the forward.  Here the only HBM traffic is h1
// (read once), the L2-resident weights and p.
//
// The split arithmetic is the engine's (k_gemm.hpp kPrecS3): h = hi + mid + lo in bf16, W pre-split into
// three planes (W3 [13 steps][3][416][32], the layers' own packed planes), six products per K step in the
// same order ("smallest terms first"), so each layer's fp32 sums are those of the unfused kernels.
//
// Block = 8 waves (two per SIMD), 128 rows per row block; persistent (grid = min(row blocks, CUs)).
//   - A wave owns 16 rows of the row block and ALL 416 columns of both layers: the MFMA runs with the
//     operands swapped (D = W h^T, v_mfma_f32_16x16x32_bf16 with the weight plane as A), so a lane holds
//     4 consecutive outputs n = 16 t + 4 g .. + 3 of sample r16 for column tile t.  Those are exactly the
//     K values lane group g needs at positions 4 h + q of the next layer's K step (the split engine's K
//     order: step c, half h, K = 32 c + 16 h + 4 g + q), so h2 = ReLU(acc2 + b2) IS layer 3's B operand,
//     in place: 25 tiles x 4 fp32 = 100 registers.
//   - h1 streams from HBM by LDS-DMA into two per-wave step slots (the wave's 16 rows x 128 B), two
//     units ahead of its use; only the issuing wave reads them.
//   - The weights stream through LDS in "units" of one K step x one column half (13 tiles x 3 planes x
//     1 KiB = 39 KiB): a 3-slot ring, unit U + 2's DMAs issued during unit U (one per column tile, so a
//     DMA's issue stall overlaps MFMAs), one barrier per unit.  A row block is 52 units: layer 2 as
//     (step c, half 0), (c, half 1) for c = 0..12 (the split h1 step feeds both halves), then layer 3 as
//     half 0's 13 steps and half 1's 13 steps (13 accumulator tiles live at a time: h2 stays live).
//     The weight units do not depend on the row block, so the ring runs on across row blocks without
//     a drain.
//   - Every wave issues the same vector-memory instructions every unit (5 weight DMAs; plus 2 h1 DMAs,
//     issued before them, in every layer-2 half-0 unit and in unit 50), so each unit's wait for its own
//     DMAs is a compile-time vmcnt.  (h1 went through registers first: the compiler's waitcnt insertion
//     then drained vmcnt(0) at the layer-2 loop head, which took the weight DMAs' lead.)
// MFMA work per row block per wave: 2 layers x 13 steps x 25 tiles x 6 = 3,900 MFMAs (tile 25, columns
// 400 .. 415, is padding in both layers and is not computed).
#include "k_rowown.hpp"

namespace rmx {
namespace {
using namespace rowown;

constexpr int kQKS = 13;                     // 32-wide K steps (Kpad = 416)
constexpr int kQUnits = 4 * kQKS;            // units per row block (52)
constexpr int kQL3 = 2 * kQKS;               // first layer-3 unit (26)
constexpr int kQPrm = 3 * kQN;               // b2 | b3 | wo (fp32) in LDS
constexpr int kQH1 = kQW * 2 * 2048;         // h1: two 2-KiB step slots per wave
constexpr size_t kQLds = (size_t)kQSlots * kQUnit + kQH1 + sizeof(float) * kQPrm;
static_assert(kQLds <= 160 * 1024, "LDS budget");

#ifndef RMX_QTAIL_PRIO
#define RMX_QTAIL_PRIO 0
#endif
// weight-fragment prefetch depth (column tiles) of the layer-3 units, where h2's 100 registers are live
#ifndef RMX_QTAIL_PF3
#define RMX_QTAIL_PF3 1
#endif

// a zero h1 row: the load source of rows past M (every lane issues the same loads at every K offset)
__device__ __attribute__((aligned(16))) float g_qzero_row[kQN];

struct TailS3Args {
  int M;
  QRows rows;  // full / half row blocks (k_rowown.hpp)
  const float* H;  // layer input [M][lda] fp32 (columns >= 400 read as zero)
  int lda;
  const bf16_t* W2;  // [13][3][416][32] bf16 planes (DenseLayer::W3)
  const float* b2;   // [416]
  const bf16_t* W3;
  const float* b3;
  OutArgs oa;  // wo [416], bo, pre, pre2, rowsum, beta, out
};

// unit u of a row block -> its weight planes, K step and column half (wave-uniform)
__device__ __forceinline__ const bf16_t* q_unit_src(const TailS3Args& p, int u) {
  const bool l3 = u >= kQL3;
  const int v = l3 ? u - kQL3 : u;
  const int half = l3 ? (v >= kQKS ? 1 : 0) : (v & 1);
  const int c = l3 ? (v >= kQKS ? v - kQKS : v) : (v >> 1);
  return (l3 ? p.W3 : p.W2) + (int64_t)(c * 3 * kQN + half * kQUT * 16) * 32;
}

// h1 of K step c of row block rb into this wave's LDS slot ds (c & 1; 2 DMA instructions: the wave's 16 rows x
// 128 B; rows past M read the zero row).  Instruction i, lane L: row r = 8 i + (L >> 3), physical 16-B
// slot L & 7, which holds logical slot j = (L & 7) ^ (r & 7), i.e. columns 32 c + 4 j .. + 3 (j < 4:
// the fragment's a0 part, j >= 4: a1).  Only the issuing wave reads these rows: its own vmcnt orders
// them, no barrier.
__device__ __forceinline__ void q_h1_dma(const TailS3Args& p, const float* zrow, char* hlds, int row0, int nw, int c,
                                         int ds, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int r = 8 * i + (lane >> 3), j = (lane & 7) ^ ((lane >> 3) & 7);
    asm volatile("" : "+v"(r), "+v"(j));  // formed here (not hoisted)
    // branch-free (an exec-masked address branch split the unit into basic blocks): rows past M
    // read the zero row at the same column offset (M * lda < 2^31: launch check)
    const int m = row0 + w * 16 + r;
    const uint32_t ok = (w < nw && m < p.M) ? 1u : 0u;
    const uintptr_t base = (uintptr_t)zrow + (uintptr_t)ok * ((uintptr_t)p.H - (uintptr_t)zrow);
    const float* row = reinterpret_cast<const float*>(base) + (uint32_t)(m * (int)ok) * (uint32_t)p.lda;
    lds_dma<16>(row + 32 * c + 4 * j, hlds + ds * 2048 + i * 1024);
  }
}
// the h1 fragment of step c from the wave's slot: a0 = columns 32 c + 4 g .., a1 = 32 c + 16 + 4 g ..
// (zero at step 12: columns 400 .. are padding)
__device__ __forceinline__ void q_h1_read(const char* hlds, int c, int lane, f32x4& a0, f32x4& a1) {
  const int r = lane & 15, g = lane >> 4;
  int o0 = r * 128 + ((g ^ (r & 7)) << 4), o1 = r * 128 + (((g + 4) ^ (r & 7)) << 4);
  asm volatile("" : "+v"(o0), "+v"(o1));
  a0 = *reinterpret_cast<const f32x4*>(hlds + (c & 1) * 2048 + o0);
  a1 = *reinterpret_cast<const f32x4*>(hlds + (c & 1) * 2048 + o1);
  if (c == kQKS - 1) a1 = f32x4{0.f, 0.f, 0.f, 0.f};
}


// layer-3 half HF (column tiles 13 HF .. + 12; half 1 computes 12, tile 25 is padding): 13 units, one
// per K step, unrolled so that h2's tiles 2c, 2c + 1 are static registers.  Unit 50 (half 1, step 11)
// also loads the next row block's h1 step 0.
template <int HF>
__device__ __forceinline__ void q_layer3(const TailS3Args& p, char* lds, const float* prm, f32x4 (&h2)[kQNT], int& slot,
                                         int w, int lane, int lo, int fb, const float* zrow, char* hlds, int it,
                                         float& part) {
  const int g = lane >> 4;
  f32x4 acc[kQUT];
#pragma unroll
  for (int t = 0; t < kQUT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < kQKS; ++c) {
    constexpr int kBase = kQL3 + HF * kQKS;
    const int u = kBase + c;
    if (u == kQUnits - 1)
      q_enter<7>();  // unit 50 issued the next block's h1 loads
    else
      q_enter<5>();
    bf16x8 ah, am, al;
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    split3(h2[2 * c], 2 * c + 1 < kQNT ? h2[2 * c + 1] : z, ah, am, al);
    if (u == kQUnits - 2) {  // the next row block's step 0 (two units ahead of its first use)
      int row0n, nwn;  // the next row block's (formed here: live across layer 3 it spilled)
      p.rows.desc(blockIdx.x, it + 1, row0n, nwn);
      q_h1_dma(p, zrow, hlds, row0n, nwn, 0, 0, w, lane);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int u2 = u + 2 >= kQUnits ? u + 2 - kQUnits : u + 2;
    const int dslot = slot == 0 ? 2 : slot - 1;  // (slot + 2) mod 3
    const char* ub = lds + slot * kQUnit;
    if constexpr (HF == 0)
      q_unit<kQUT, 0, kQUT, RMX_QTAIL_PF3>(ub, fb, ah, am, al, acc, q_unit_src(p, u2), lds, dslot, w, lo);
    else
      q_unit<kQUT - 1, 0, kQUT, RMX_QTAIL_PF3>(ub, fb, ah, am, al, acc, q_unit_src(p, u2), lds, dslot, w, lo);
    slot = q_next(slot);
  }
  // the output dot over this half's columns: ReLU(acc + b3)[n] * wo[n], n = 16 (13 HF + t) + 4 g + q
  constexpr int NT = HF == 0 ? kQUT : kQNT - kQUT;
  __builtin_amdgcn_sched_barrier(0);  // (the epilogue's LDS reads hoisted into the last unit spilled)
  int g4 = 4 * g;
  asm volatile("" : "+v"(g4));  // (the 2 x 13 LDS addresses formed here, not hoisted into spills)
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n0 = 16 * (kQUT * HF + t) + g4;
    const f32x4 bb = *reinterpret_cast<const f32x4*>(prm + kQN + n0);
    const f32x4 wv = *reinterpret_cast<const f32x4*>(prm + 2 * kQN + n0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = acc[t][r] + bb[r];
      v = v > 0.f ? v : 0.f;
      part += v * wv[r];
    }
  }
  // the dot is done here: sunk to its use after half 1, it kept half 0's 13 accumulators alive and spilled
  asm volatile("" : "+v"(part));
}

// A row block without MFMAs, for a wave that owns no rows in it (QRows half blocks): the same 52 units,
// barriers and vector-memory instructions as the computing waves (h1 loads of zero rows included), so
// the ring and every static vmcnt count stay in step.
__device__ __forceinline__ void q_idle_block(const TailS3Args& p, char* lds, int& slot, int w, int lane, int lo,
                                             const float* zrow, char* hlds, int it, int row0, int nw) {
#pragma unroll 1
  for (int c = 0; c < kQKS; ++c) {
    q_enter<5>();
    q_h1_dma(p, zrow, hlds, row0, nw, c + 1 < kQKS ? c + 1 : c, (c + 1) & 1, w, lane);
    __builtin_amdgcn_sched_barrier(0);
    int dslot = slot == 0 ? 2 : slot - 1;
    q_dma_only(q_unit_src(p, 2 * c + 2), lds, dslot, w, lo);
    slot = q_next(slot);
    q_enter<7>();
    dslot = slot == 0 ? 2 : slot - 1;
    q_dma_only(q_unit_src(p, 2 * c + 3), lds, dslot, w, lo);
    slot = q_next(slot);
  }
#pragma unroll 1
  for (int u = kQL3; u < kQUnits; ++u) {
    if (u == kQUnits - 1)
      q_enter<7>();
    else
      q_enter<5>();
    if (u == kQUnits - 2) {
      int row0n, nwn;
      p.rows.desc(blockIdx.x, it + 1, row0n, nwn);
      q_h1_dma(p, zrow, hlds, row0n, nwn, 0, 0, w, lane);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int u2 = u + 2 >= kQUnits ? u + 2 - kQUnits : u + 2;
    const int dslot = slot == 0 ? 2 : slot - 1;
    q_dma_only(q_unit_src(p, u2), lds, dslot, w, lo);
    slot = q_next(slot);
  }
}

__global__ __launch_bounds__(kQThreads, 1) void tower_tail_s3_kernel(TailS3Args p) {
  extern __shared__ __attribute__((aligned(16))) char qsmem[];
  char* lds = qsmem;
  float* prm = reinterpret_cast<float*>(qsmem + kQSlots * kQUnit + kQH1);  // b2 | b3 | wo
  const float* zrow = g_qzero_row;
  asm volatile("" : "+s"(zrow));
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
#if RMX_QTAIL_PRIO
  if (w >= kQW / 2) __builtin_amdgcn_s_setprio(1);  // (timing A/B) the second-dispatched half at priority 1
#endif
  const int nit = p.rows.nit(blockIdx.x);
  const OutArgs& oa = p.oa;

  for (int i = tid; i < kQPrm; i += kQThreads) {
    const int a = i / kQN, n = i - a * kQN;
    const float* src = a == 0 ? p.b2 : (a == 1 ? p.b3 : oa.wo);
    prm[i] = src ? src[n] : 0.f;
  }
  // lane offset of the DMA sources: row L >> 2 of a tile, logical slot swz_slot(row, L & 3), 8 bf16 each
  int lo = (lane >> 2) * 32 + swz_slot(lane >> 2, lane & 3) * 8;
  asm volatile("" : "+v"(lo));
  const int fb = q_fbase(lane);

  char* hlds = qsmem + kQSlots * kQUnit + w * 4096;  // this wave's h1 step slots
  {
    int row0, nw;
    p.rows.desc(blockIdx.x, 0, row0, nw);
    q_h1_dma(p, zrow, hlds, row0, nw, 0, 0, w, lane);
  }
  if (nit > 0) {
    const bf16_t* s0 = q_unit_src(p, 0);
    const bf16_t* s1 = q_unit_src(p, 1);
#pragma unroll
    for (int q = 0; q < kQQ; ++q) q_dma(s0, lds, 0, w, q, lo);
#pragma unroll
    for (int q = 0; q < kQQ; ++q) q_dma(s1, lds, 1, w, q, lo);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // prm staged; units 0 and 1 (this wave's) landed -- q_enter's barrier covers the rest

  int slot = 0;
  for (int it = 0; it < nit; ++it) {
    int row0, nw;
    p.rows.desc(blockIdx.x, it, row0, nw);
    if (w >= nw) {  // a half block's waves 4 .. 7: the ring only (one branch per row block: per-unit
      q_idle_block(p, lds, slot, w, lane, lo, zrow, hlds, it, row0, nw);  // branches spilled)
      continue;
    }
    // ---- layer 2: units (c, half 0), (c, half 1) ----
    f32x4 h2[kQNT];
#pragma unroll
    for (int t = 0; t < kQNT; ++t) h2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int c = 0; c < kQKS; ++c) {
      q_enter<5>();  // previous unit: (c - 1, half 1) or the last layer-3 unit, 5 DMAs
      bf16x8 ah, am, al;
      {
        f32x4 a0, a1;
        q_h1_read(hlds, c, lane, a0, a1);
        split3(a0, a1, ah, am, al);
      }
      // the next step's h1 (two units ahead of its use; at c = 12 a harmless reload of step 12 into slot 1,
      // which is next written by the next row block's step 1)
      q_h1_dma(p, zrow, hlds, row0, nw, c + 1 < kQKS ? c + 1 : c, (c + 1) & 1, w, lane);
      __builtin_amdgcn_sched_barrier(0);  // the h1 loads ahead of this unit's DMAs (the static vmcnt counts)
      const int u = 2 * c;
      int dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kQUT, 0>(lds + slot * kQUnit, fb, ah, am, al, h2, q_unit_src(p, u + 2), lds, dslot, w, lo);
      slot = q_next(slot);
      q_enter<7>();  // previous unit issued 2 h1 loads + 5 DMAs
      dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kQNT - kQUT, kQUT>(lds + slot * kQUnit, fb, ah, am, al, h2, q_unit_src(p, u + 3), lds, dslot, w, lo);
      slot = q_next(slot);
    }
    // h2 = ReLU(acc2 + b2), in place
    __builtin_amdgcn_sched_barrier(0);
    int g4 = 4 * g;
    asm volatile("" : "+v"(g4));
#pragma unroll
    for (int t = 0; t < kQNT; ++t) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(prm + 16 * t + g4);
      h2[t] = relu4(h2[t] + bb);
    }
    // ---- layer 3 + the output dot ----
    float part = 0.f;
    q_layer3<0>(p, lds, prm, h2, slot, w, lane, lo, fb, zrow, hlds, it, part);
    q_layer3<1>(p, lds, prm, h2, slot, w, lane, lo, fb, zrow, hlds, it, part);
    // ---- head: the four lane groups' columns, then bias, CAddTable, sigmoid (out_finish_kernel's order) ----
    part += __shfl_xor(part, 16);
    part += __shfl_xor(part, 32);
    const int m = row0 + w * 16 + r16;
    if (g == 0 && m < p.M) {
      float y = part;
      if (oa.has_bo) y = y + oa.bo;
      if (oa.rowsum) {
        float rs = 0.f;
        for (int jj = 0; jj < oa.rowsum_k; ++jj) rs += oa.rowsum[(int64_t)m * oa.rowsum_k + jj];
        y = rs + y;
      }
      if (oa.pre2) y = oa.pre2[m] + y;
      float tt = oa.pre ? oa.pre[m] + y : y;
      tt = tt + oa.beta;
      oa.out[m] = 1.0f / (1.0f + expf(-tt));
    }
  }
  // the ring's trailing DMAs (units 0 / 1 of a row block that does not exist) land before the block's
  // LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

bool tower_tail_s3_usable(const DenseLayer& L2, const DenseLayer& L3, int M, int lda) {
  if (M <= 0 || !L2.W3 || !L3.W3 || L2.W16 || L3.W16 || !f32_split_enabled()) return false;
  // (Kpad is the fp32 packing's multiple of 16: 400; its split planes hold ceil(25 / 2) = 13 K steps)
  if (!(L2.K == 400 && L2.N == 400 && L3.K == 400 && L3.N == 400 && L2.Npad == kQN && L3.Npad == kQN &&
        (L2.Kpad + 31) / 32 == kQKS && (L3.Kpad + 31) / 32 == kQKS && L2.N1 < 0 && L3.N1 < 0 && L2.bias_mode == 1 && L3.bias_mode == 1 &&
        lda >= kQN && lda % 4 == 0))
    return false;
  // knob "s3_tail": 0 off, 2 always, 1 (default) when the (half) row blocks fill every CU at least once
  const int knob = tuning_get("s3_tail", 1);
  if (knob == 0) return false;
  if (knob == 2) return true;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  // (half) row blocks that fill every CU, or -- with half blocks -- any batch above the whole-tower kernel's
  // one round (k_small_s3.hip: M <= 16 ncu): half blocks on part of the chip still beat three engine launches
  return q_fills(M, ncu) || (tuning_get("half_blocks", 1) != 0 && M > 16 * ncu);
}

int launch_tower_tail_s3(hipStream_t s, const DenseLayer& L2, const DenseLayer& L3, int M, const float* H, int lda,
                         const OutArgs& oa) {
  if (!oa.wo || !oa.out || !L2.W3 || !L3.W3 || L2.Npad != kQN || L3.Npad != kQN || L2.K != 400 || L3.K != 400 ||
      L2.N != 400 || L3.N != 400 || lda < kQN || lda % 4) {
    set_error("fp32 tower tail: needs two 400 x 400 split-GEMM layers and an output head");
    return RMX_E_INVALID;
  }
  if (M <= 0) return RMX_OK;
  if ((int64_t)M * lda >= ((int64_t)1 << 31)) {
    set_error("fp32 tower tail: batch too large for one launch");
    return RMX_E_INVALID;
  }
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  RMX_HIP(hipFuncSetAttribute((const void*)tower_tail_s3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kQLds));
  TailS3Args p{};
  p.M = M;
  int grid = 0;
  p.rows = q_rows(M, ncu, grid);
  p.H = H;
  p.lda = lda;
  p.W2 = L2.W3;
  p.b2 = L2.b;
  p.W3 = L3.W3;
  p.b3 = L3.b;
  p.oa = oa;
  hipLaunchKernelGGL(tower_tail_s3_kernel, dim3(grid), dim3(kQThreads), kQLds, s, p);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
