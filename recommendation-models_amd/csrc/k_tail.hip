// k_tail.hip -- the bf16 tower tail in one persistent kernel (BASELINE.json configs[4]: DCN / PNN
// bf16, gfx950).
//
// The last hidden Linear + ReLU and the output Linear + head of a bf16 tower
// (model/encoder/HigherOrderEncoder.scala:34-59: Linear(400 -> 400) + ReLU, then the last
// Linear(400 -> 400) + ReLU whose output feeds Linear(400 -> 1); the heads of DCN.scala /
// PNN.scala: CAddTable + Sigmoid) as ONE launch over row blocks of 128 samples:
//   h2 = bf16(ReLU(h1 W2^T + b2))        kept in LDS, never written to HBM
//   y  = sum_n ReLU(h2 W3^T + b3)[n] wo[n] (+ bo) ; p = sigmoid(pre + (pre2 + y) + beta)
// Why: run as two launches, each layer reads 52 MB and the first writes 52 MB at B = 65,536, with
// one stage of 30 KiB in flight per block (26 KiB of it the weights from L2), so both layers sat
// at ~2.9 TB/s and 0.2 of the bf16 peak, bound by memory latency rather than by HBM or MFMA.
// Here the only HBM traffic is h1 (read once) and p.
//
// Block = 16 waves on one CU (persistent: grid = min(row blocks, CUs)):
//   - 3 loader waves DMA the NEXT row block's h1 tile (128 rows x 416 bf16 = 104 KiB, global_load_lds)
//     into rotating LDS step slots while the 13 compute waves run the current one (slot map and
//     schedule below), so the tile's HBM latency hides behind the MFMAs (a loader's vmcnt wait stalls
//     only the loader: every wave has its own counter); loader 0 also runs each block's head;
//   - compute wave w < 12 owns column tiles w, w + 12 of both layers for all 128 rows, wave 12 tile 24
//     (the 25 tiles of N = 400): 7 / 6 / 6 / 6 tiles per SIMD (waves w and w + 4 share a SIMD);
//   - the weights (W2, W3: [13 steps][416][32] bf16, 338 KiB each, L2-resident) go straight from
//     global memory into registers, one K step ahead: each fragment is 1 KiB contiguous per wave
//     and exactly one wave of the block reads it, so staging it through LDS would buy no reuse;
//   - the MFMA runs with the operands swapped (D = W h^T: v_mfma_f32_16x16x32_bf16 with the weight
//     fragment as A), so a lane ends up holding 4 consecutive outputs n of one sample, which is
//     what the epilogue needs: h2 goes back into the block's own LDS slots as one 8-B bf16x4 write
//     per (tile, row tile), and the output dot sums along the lane first.
// Per K step a compute wave reads 8 h fragments (8 KiB) from LDS and issues 8 x NTW MFMAs: each weight
// fragment feeds 8 MFMAs (at 64 rows per block the weight stream was half the kernel's time).
// The sums are the unfused kernels' up to the order of the final logit reduction: h2 is the same
// bf16 (RNE) of the same fp32 accumulations (K steps in order), so parity is held to the same bar
// against the oracle's bf16 emulation (tests/test_bf16.py).
// LDS DMAs through the builtin in this translation unit (k_gemm.hpp lds_dma): measured faster here than
// the asm form, bf16 tail 0.042 vs 0.048 ms with the asm form (profiles/r04/ab_lds_dma_form.txt)
#define RMX_LDS_DMA_BUILTIN 1
#include "k_gemm.hpp"

namespace rmx {
namespace {

constexpr int kTBM = 128;                  // rows per row block
constexpr int kTMT = kTBM / 16;            // row tiles
constexpr int kTNT = 25;                   // computed 16-column tiles (N <= 400)
constexpr int kTN = 416;                   // Npad: packed rows of W per K step
constexpr int kTKS = 13;                   // 32-wide K steps: Kpad = 416
constexpr int kTCW = 13;                   // compute waves: w < 12 own tiles w, w + 12; wave 12 tile 24
constexpr int kTLW = 3;                    // loader waves (13, 14, 15)
constexpr int kTThreads = (kTCW + kTLW) * 64;
constexpr int kTStep = kTBM * 64;         // bytes of one K step of a row block's h tile (8 KiB)
constexpr int kTSlots = 18;                // LDS step slots: 13 of the current row block + 5 spare
constexpr int kTImg = kTSlots * kTStep;    // 147,456 B
constexpr int kTE = 5;                     // "early" K steps of a row block (loaded a whole row block ahead)
constexpr int kTL3 = kTKS - kTE;           // layer-3 steps read before the slots of the next block's late steps free up (8)
constexpr int kTInsE = kTE * kTStep / 1024;            // 1-KiB DMA instructions: early steps (40)
constexpr int kTInsL = (kTKS - kTE) * kTStep / 1024;   // late steps (64)
// weight fragments loaded this many K steps ahead: 1 (2 spilled 14 registers at the 128-VGPR budget of
// 16 waves: tail 0.0463 vs 0.0443 ms, 11.3 vs 5.0 MB of scratch writes per launch)
constexpr int kTPF = 1;
constexpr int kTPrm = 3 * kTN;              // b2, b3, wo staged in LDS (fp32)
constexpr size_t kTLds = kTImg + sizeof(float) * (kTCW * kTBM + kTPrm);

static_assert(kTLds <= 160 * 1024, "LDS budget");
static_assert(kTSlots == kTKS + kTE && kTL3 == kTKS - kTE, "the slot rotation below");
static_assert(kTInsE == 40 && kTInsL == 64 && kTLW == 3,
              "the loaders' counted vmcnt waits: 40 early-step DMAs (14 / 13 / 13), 64 late ones (22 / 21 / 21)");

// The 18 step slots rotate between row blocks: block t holds its K step c in slot S_t[c].  Block t + 1's
// early steps go to the 5 slots block t does not use (loadable any time during block t), its late steps
// (5 .. 12) to block t's steps 0 .. 7, free once layer 3 of block t has read them:
//   S_{t+1}[0..4] = F_t,  S_{t+1}[5..12] = S_t[0..7],  F_{t+1} = S_t[8..12];  S_0 = 0..12, F_0 = 13..17.
// S_t ++ F_t is then [0..17] rotated right by 5 t, i.e. S_t[c] = (c + base_t) mod 18 with base_0 = 0 and
// base_{t+1} = base_t + 13 mod 18: one wave-uniform integer per block (a table of 18 slots per block was
// kept in scratch by the compiler).  The early steps have a whole row block of lead and the late ones
// layer 3's last 5 steps + layer 2's first 5 (the previous two-half image gave each half about half a
// layer, and layer 2 waited at its mid barrier).
struct SlotMap {
  int base;
};
__device__ __forceinline__ SlotMap slots_first() { return SlotMap{0}; }
__device__ __forceinline__ SlotMap slots_next(const SlotMap& m) {
  const int b = m.base + kTKS;
  return SlotMap{b >= kTSlots ? b - kTSlots : b};
}
// slot of step c (c < 13, wave-uniform)
__device__ __forceinline__ int slot_at(const SlotMap& m, int c) {
  const int s = c + m.base;
  return s >= kTSlots ? s - kTSlots : s;
}

// Diagnostic builds only (timing probes, wrong results; never set in librmx.so): 1 = no weight loads
// in the K loops (the prologue's fragments reused), 4 = no h1 prefetch after the first tile, 8 = no
// head (the finish of each row block)
#ifndef RMX_TAIL_DIAG
#define RMX_TAIL_DIAG 0
#endif
// 16: s_memtime stamps of block 0's waves 0, 2, 12 (compute) and 13 (loader 0) at every barrier of
// its row blocks (tools/diag_tail_stamps.py reads them through rmx_diag_tail)
#if RMX_TAIL_DIAG & 16
__device__ unsigned long long g_tail_t[4][40];
#define TS(k)                                                                              \
  do {                                                                                     \
    if (dslot >= 0 && (k) < 40) g_tail_t[dslot][k] = __builtin_amdgcn_s_memtime();       \
  } while (0)
#else
#define TS(k) \
  do {        \
  } while (0)
#endif

struct TailArgs {
  int M, nblk;
  const bf16_t* H;  // layer input [M][lda] bf16; columns >= K2 read as zero
  int lda, K2;
  const bf16_t* W2;  // [13][416][32]
  const float* b2;   // [416]
  const bf16_t* W3;
  const float* b3;
  OutArgs oa;        // wo [416], bo, pre, pre2, rowsum, beta, out
  // first order computed here instead of read from oa.pre (PNN: its own kernel otherwise): y1[m] =
  // sum_f w[ids[m * F + f] * wld] in field order (encoder_k16_kernel<0>'s sum), null = off
  const int32_t* fo_ids;
  const bf16_t* fo_w;
  int fo_F, fo_wld;
};

__device__ __forceinline__ void bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// weight fragment of K step c, the wave's column tile j: lane offset wo = this lane's element of the
// wave's first tile ((w * 16 + r16) * 32 + g * 8); tile j is 12 tiles further: 1 KiB per wave.  W stays
// a kernel-argument pointer (global address space: global_load, counted by vmcnt only; a laundered
// pointer would become a flat load, which also counts in lgkmcnt and made every LDS wait a full drain)
__device__ __forceinline__ f32x4 ldw(const bf16_t* __restrict__ W, int wo, int c, int j) {
  return *reinterpret_cast<const f32x4*>(W + wo + (c * kTN + j * 12 * 16) * 32);
}
// the lane's offset for ldw, opaque to the optimiser so that the fragment addresses are formed step
// by step instead of being hoisted out of the row-block loop (which spilled)
__device__ __forceinline__ int wlane(int w, int lane) {
  int wo = (w * 16 + (lane & 15)) * 32 + (lane >> 4) * 8;
  asm volatile("" : "+v"(wo));
  return wo;
}
// h fragment of K step c, row tile i, from the swizzled image.  The swizzle key of row 16 i + r16 is
// that of r16 ((row >> 2) & 3 drops the 16 i), so a lane's fragments sit at one per-lane base hb =
// (r16 * 4 + swz_slot(r16, g)) * 16 plus compile-time offsets (ds_read immediates); hb is opaque so
// the 13 x 8 addresses are not formed up front (they spilled)
__device__ __forceinline__ int hbase(int lane) {
  int hb = ((lane & 15) * 4 + swz_slot(lane & 15, lane >> 4)) * 16;
  asm volatile("" : "+v"(hb));
  return hb;
}
__device__ __forceinline__ f32x4 ldh(const char* img, int hb, int slot, int i) {
  return *reinterpret_cast<const f32x4*>(img + slot * kTStep + hb + i * 1024);
}

// K steps [C0, C1) of a layer: acc[i][j] (row tile i, column tile j) += W_j h_i^T; wb holds the
// fragments of steps C0 .. C0 + kTPF - 1 on entry (ring slot c % (kTPF + 1))
template <int NTW, int C0, int C1>
__device__ __forceinline__ void tail_steps(const bf16_t* __restrict__ W, int wo, const char* img, const SlotMap& sm,
                                           int lane, f32x4 (&acc)[kTMT][NTW], f32x4 (&wb)[kTPF + 1][NTW]) {
  const int hb = hbase(lane);
#pragma unroll
  for (int c = C0; c < C1; ++c) {
    if (c + kTPF < kTKS && !(RMX_TAIL_DIAG & 1)) {
      int wc = wo + (c + kTPF) * kTN * 32;
      asm volatile("" : "+v"(wc));  // formed here, not all 13 at the layer's start
#pragma unroll
      for (int j = 0; j < NTW; ++j) wb[(c + kTPF) % (kTPF + 1)][j] = ldw(W, wc, 0, j);
    }
    // two groups of four row tiles: each group's four fragments, then its MFMAs (all eight at
    // once would hold 32 more registers)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4 a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = ldh(img, hb, slot_at(sm, c), 4 * h + i);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j)
          acc[4 * h + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, wb[c % (kTPF + 1)][j]), __builtin_bit_cast(bf16x8, a[i]), acc[4 * h + i][j], 0, 0, 0);
    }
  }
}

template <int NTW>
__device__ __forceinline__ void tail_prologue(const bf16_t* __restrict__ W, int wo, f32x4 (&wb)[kTPF + 1][NTW]) {
#pragma unroll
  for (int c = 0; c < kTPF; ++c)
#pragma unroll
    for (int j = 0; j < NTW; ++j) wb[c][j] = ldw(W, wo, c, j);
}

template <int NTW>
__device__ __forceinline__ void tail_zero(f32x4 (&acc)[kTMT][NTW]) {
#pragma unroll
  for (int i = 0; i < kTMT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// h2 columns n0 .. n0 + 3 of rows 16 i + r16 go to per-lane base pbase(n0) + 1 KiB * i (same key
// argument as hbase) as one bf16x4 (8 B)
// (the K step n0 >> 5 of a column tile is wave-uniform: its step slot goes into the base)
__device__ __forceinline__ int pbase(int lane, int n0, const SlotMap& sm) {
  const int r16 = lane & 15, c = n0 >> 5, q = (n0 & 31) >> 3, half = (n0 >> 2) & 1;
  int pb = slot_at(sm, __builtin_amdgcn_readfirstlane(c)) * kTStep + (r16 * 4 + swz_slot(r16, q)) * 16 + half * 8;
  asm volatile("" : "+v"(pb));
  return pb;
}
__device__ __forceinline__ void put_h2(char* img, int pb, int i, const f32x4& v) {
  *reinterpret_cast<bf16x4*>(img + pb + i * 1024) = __builtin_convertvector(v, bf16x4);
}

// the fused first order of row m: all F ids, then all F weights in flight (two latency rounds), summed in
// field order from 0 (encoder_k16_kernel<0>'s y1, bitwise).  FF compile-time (no per-field conditions:
// with a runtime F they became 40 scalar masks and spilled); fo_sum_any: 8 fields at a time
template <int FF>
__device__ __forceinline__ float fo_sum(const TailArgs& p, int m) {
  int idv[FF];
#pragma unroll
  for (int f = 0; f < FF; ++f) idv[f] = p.fo_ids[(int64_t)m * FF + f];
  float wv[FF];
#pragma unroll
  for (int f = 0; f < FF; ++f) wv[f] = (float)p.fo_w[(int64_t)idv[f] * p.fo_wld];
  float y1 = 0.f;
#pragma unroll
  for (int f = 0; f < FF; ++f) y1 += wv[f];
  return y1;
}
__device__ __forceinline__ float fo_sum_any(const TailArgs& p, int m) {
  float y1 = 0.f;
#pragma unroll 1
  for (int f0 = 0; f0 < p.fo_F; f0 += 8) {
    float wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      wv[u] = f0 + u < p.fo_F ? (float)p.fo_w[(int64_t)p.fo_ids[(int64_t)m * p.fo_F + f0 + u] * p.fo_wld] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (f0 + u < p.fo_F) y1 += wv[u];
  }
  return y1;
}

// issuing wave idx of nidx: its share of K steps [C0, C1) of row block rb's h1 tile into the step slots
// of map sm (8 1-KiB DMA instructions per step).  Lane L of instruction q of a step fills tile row
// 16 q + L / 4 at physical 16-B slot L & 3, i.e. loads logical slot swz_slot(row, L & 3) (the swizzle is
// an involution).
template <int C0, int C1>
__device__ __forceinline__ void tail_issue(const TailArgs& p, char* img, const SlotMap& sm, int rb, int idx, int nidx,
                                           int lane, const float* zero16) {
  constexpr int nins = (C1 - C0) * kTStep / 1024;
  const int m0 = rb * kTBM;
  // a rolled loop: unrolled, the per-lane sources / LDS bases were formed up front and spilled
#pragma unroll 1
  for (int k = idx; k < nins; k += nidx) {
    const int c = C0 + (k >> 3), q = k & 7;
    const int row = q * 16 + (lane >> 2);
    const int m = m0 + row, kk = c * 32 + swz_slot(row, lane & 3) * 8;
    const void* src = (m < p.M && kk < p.K2) ? (const void*)(p.H + (int64_t)m * p.lda + kk) : (const void*)zero16;
    char* dst = img + slot_at(sm, c) * kTStep + q * 1024;
    lds_dma<16>(src, dst);
  }
}

// Compute wave with first column tile w (NTW tiles: w, w + 12; the last compute wave w = 24, one
// tile): barriers B0, BM2, B1, B2, BM3, B3 per row block, the same six as the loaders
template <int NTW>
__device__ void tail_compute(const TailArgs& p, char* img, float* red, const float* prm, int w, int lane, int nit,
                             const float* zero16) {
  const int g = lane >> 4, r16 = lane & 15;
#if RMX_TAIL_DIAG & 16
  const int dslot = (blockIdx.x == 0 && lane == 0) ? (w == 0 ? 0 : (w == 2 ? 1 : (w == 24 ? 2 : -1))) : -1;
#endif
  TS(0);
  f32x4 acc[kTMT][NTW];
  f32x4 wb[kTPF + 1][NTW];
  SlotMap sm = slots_first();
  // the first row block's early steps: every wave of the block issues its DMAs (issue, not HBM, limits a
  // start from an empty image), then the weight prologue
  if (nit > 0) tail_issue<0, kTE>(p, img, sm, blockIdx.x, w < 12 ? w : kTCW - 1, 16, lane, zero16);
  tail_prologue<NTW>(p.W2, wlane(w, lane), wb);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int it = 0; it < nit; ++it) {
    bar();  // B0: this row block's early steps have landed
    TS(1 + 10 * it);
    {
      const int wo = wlane(w, lane);
      tail_zero<NTW>(acc);
      tail_steps<NTW, 0, kTE>(p.W2, wo, img, sm, lane, acc, wb);
      TS(2 + 10 * it);
      bar();  // BM2: its late steps have landed
      TS(3 + 10 * it);
      tail_steps<NTW, kTE, kTKS>(p.W2, wo, img, sm, lane, acc, wb);
    }
    tail_prologue<NTW>(p.W3, wlane(w, lane), wb);  // in flight across the epilogue
    TS(4 + 10 * it);
    bar_lds();                                      // B1: every wave has read the h1 tile
    TS(5 + 10 * it);
    // h2 = bf16(ReLU(acc + b2)) into the same slots; lane holds n = 16 t + 4 g .. + 3 of row 16 i + r16
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n0 = 16 * (w + 12 * j) + 4 * g;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(prm + n0);
      const int pb = pbase(lane, n0, sm);
#pragma unroll
      for (int i = 0; i < kTMT; ++i) {
        f32x4 v = acc[i][j] + bb;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
        put_h2(img, pb, i, v);
      }
    }
    if (w == 2 * 12) {  // columns 400 .. 415 (not computed) read as zeros by the next layer
      const int pb = pbase(lane, 16 * kTNT + 4 * g, sm);
#pragma unroll
      for (int i = 0; i < kTMT; ++i) put_h2(img, pb, i, f32x4{0.f, 0.f, 0.f, 0.f});
    }
    bar_lds();  // B2: h2 complete
    TS(6 + 10 * it);
    {
      const int wo = wlane(w, lane);
      tail_zero<NTW>(acc);
      tail_steps<NTW, 0, kTL3>(p.W3, wo, img, sm, lane, acc, wb);
      TS(7 + 10 * it);
      bar_lds();  // BM3: steps 0 .. 7 read by every wave: the loaders refill them with the next block
      TS(8 + 10 * it);
      tail_steps<NTW, kTL3, kTKS>(p.W3, wo, img, sm, lane, acc, wb);
    }
    if (it + 1 < nit) tail_prologue<NTW>(p.W2, wlane(w, lane), wb);
    // output dot: part[i] = sum over this lane's n of ReLU(acc + b3)[n] * wo[n], then over the 4 lane groups
    float part[kTMT];
#pragma unroll
    for (int i = 0; i < kTMT; ++i) part[i] = 0.f;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n0 = 16 * (w + 12 * j) + 4 * g;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(prm + kTN + n0);
      const f32x4 wv = *reinterpret_cast<const f32x4*>(prm + 2 * kTN + n0);
#pragma unroll
      for (int i = 0; i < kTMT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bb[r];
          v = v > 0.f ? v : 0.f;
          part[i] += v * wv[r];
        }
    }
#pragma unroll
    for (int i = 0; i < kTMT; ++i) {
      part[i] += __shfl_xor(part[i], 16);
      part[i] += __shfl_xor(part[i], 32);
      if (g == 0) red[(w < 12 ? w : kTCW - 1) * kTBM + 16 * i + r16] = part[i];
    }
    TS(9 + 10 * it);
    bar_lds();  // B3: partial logits complete
    TS(10 + 10 * it);
    sm = slots_next(sm);
  }
}

__global__ __launch_bounds__(kTThreads, 1) void tower_tail_bf16_kernel(TailArgs p) {
  extern __shared__ __attribute__((aligned(16))) char tsmem[];
  char* img = tsmem;
  float* red = reinterpret_cast<float*>(tsmem + kTImg);  // [kTCW][kTBM] partial logits
  float* prm = red + kTCW * kTBM;                         // b2 | b3 | wo, kTN each
  const float* zero16 = g_rmx_zero16;
  asm volatile("" : "+s"(zero16));
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nit = blockIdx.x < p.nblk ? (p.nblk - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (w < kTCW - 1) {
    tail_compute<2>(p, img, red, prm, w, lane, nit, zero16);
  } else if (w == kTCW - 1) {
    tail_compute<1>(p, img, red, prm, 2 * 12, lane, nit, zero16);
  } else {
    // loaders.  Row block t + 1's early steps stream in behind row block t from BM2 on (a whole block of
    // lead), its late steps behind layer 3's last 5 steps and layer 2's first 5 of block t + 1.  Loader 0
    // also runs the head of block t - 1 after B0 (its inputs loaded a block early; red[] is rewritten
    // only after the next BM3).
    const int lw = w - kTCW;
    const OutArgs& oa = p.oa;
#if RMX_TAIL_DIAG & 16
    const int dslot = (blockIdx.x == 0 && lane == 0 && lw == 0) ? 3 : -1;
#endif
    TS(0);
    SlotMap sm = slots_first();
    if (nit > 0) tail_issue<0, kTE>(p, img, sm, blockIdx.x, kTCW + lw, 16, lane, zero16);
    {  // the epilogue parameters into LDS (read after B1 / BM3 by the compute waves)
      float v[(kTPrm + kTLW * 64 - 1) / (kTLW * 64)];
#pragma unroll
      for (int q = 0; q < (int)(sizeof(v) / sizeof(float)); ++q) {
        const int i = lw * 64 + lane + q * kTLW * 64;
        const int a = i / kTN, n = i - a * kTN;
        const float* src = a == 0 ? p.b2 : (a == 1 ? p.b3 : oa.wo);
        v[q] = (i < kTPrm && src) ? src[n] : 0.f;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (and this loader's early-step DMAs: B0 needs them)
#pragma unroll
      for (int q = 0; q < (int)(sizeof(v) / sizeof(float)); ++q) {
        const int i = lw * 64 + lane + q * kTLW * 64;
        if (i < kTPrm) prm[i] = v[q];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (nit > 0) tail_issue<kTE, kTKS>(p, img, sm, blockIdx.x, lw, kTLW, lane, zero16);
    // the head: loaders 0 and 1, one row each per lane (row = 64 lw + lane); its inputs are loaded a block
    // early (hin: pre2 or the CIN partials, hpre: pre or the fused first order)
    const bool hl = lw < 2;
    const int hrow = lw * 64 + lane;
    const bool has_pre = oa.pre || p.fo_ids;
    float hin = 0.f, hpre = 0.f, pin = 0.f, ppre = 0.f;
    auto head = [&](int rb, float in2, float pr) {
      const int m = rb * kTBM + hrow;
      if (m < p.M) {
        float y = red[hrow];
#pragma unroll
        for (int q = 1; q < kTCW; ++q) y += red[q * kTBM + hrow];
        if (oa.has_bo) y = y + oa.bo;
        if (oa.rowsum || oa.pre2) y = in2 + y;
        float t = has_pre ? pr + y : y;
        t = t + oa.beta;
        oa.out[m] = 1.0f / (1.0f + expf(-t));
      }
    };
    for (int it = 0; it < nit; ++it) {
      const int rb = blockIdx.x + it * gridDim.x;
      const SlotMap nx = slots_next(sm);
      // early steps of block it landed: only the late-step DMAs of this loader (issued after them) may be
      // in flight -- 22 for loader 0, 21 for the others (64 instructions over 3 loaders)
      if (it > 0) {
        if (lw == 0)
          asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
      }
      TS(1 + 10 * it);
      bar();  // B0
      if (it > 0 && hl && !(RMX_TAIL_DIAG & 8)) head(rb - (int)gridDim.x, pin, ppre);
      if (hl) {
        const int m = rb * kTBM + hrow;
        if (m < p.M) {
          float rs = 0.f;
          if (oa.rowsum)
            for (int jj = 0; jj < oa.rowsum_k; ++jj) rs += oa.rowsum[(int64_t)m * oa.rowsum_k + jj];
          hin = oa.rowsum ? rs : (oa.pre2 ? oa.pre2[m] : 0.f);  // (rowsum and pre2 never together)
          if (p.fo_ids) {
            hpre = p.fo_F == 39 ? fo_sum<39>(p, m) : fo_sum_any(p, m);  // (F = 39: the Criteo shape)
          } else {
            hpre = oa.pre ? oa.pre[m] : 0.f;
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // late steps landed
      TS(2 + 10 * it);
      bar();  // BM2
      // the next block's early steps into the 5 slots this block does not use
      if (it + 1 < nit && !(RMX_TAIL_DIAG & 4)) tail_issue<0, kTE>(p, img, nx, rb + gridDim.x, lw, kTLW, lane, zero16);
      bar();  // B1
      bar();  // B2
      bar();  // BM3
      // its late steps into this block's steps 0 .. 7, just read by layer 3
      if (it + 1 < nit && !(RMX_TAIL_DIAG & 4)) tail_issue<kTE, kTKS>(p, img, nx, rb + gridDim.x, lw, kTLW, lane, zero16);
      bar();  // B3
      pin = hin;
      ppre = hpre;
      sm = nx;
    }
    if (hl && nit > 0 && !(RMX_TAIL_DIAG & 8)) head(blockIdx.x + (nit - 1) * gridDim.x, pin, ppre);
  }
}

}  // namespace

#if RMX_TAIL_DIAG & 16
extern "C" int rmx_diag_tail(unsigned long long* out160) {
  return hipMemcpyFromSymbol(out160, HIP_SYMBOL(g_tail_t), sizeof(unsigned long long) * 160) == hipSuccess ? 0 : -5;
}
#endif

bool tower_tail_usable(const DenseLayer& L2, const DenseLayer& L3, int M, int lda) {
  return tuning_get("bf16_tail", 1) != 0 && M > 0 && L2.W16 && L3.W16 && L2.Npad == kTN && L3.Npad == kTN &&
         L2.N <= 16 * kTNT && L3.N <= 16 * kTNT && L2.Kpad == kTKS * 32 && L3.Kpad == kTKS * 32 &&
         L3.K <= 16 * kTNT && lda >= L2.K && lda % 8 == 0 && L2.N1 < 0 && L3.N1 < 0;
}

int launch_tower_tail_bf16(hipStream_t s, const DenseLayer& L2, const DenseLayer& L3, int M, const bf16_t* H, int lda,
                           const OutArgs& oa, const TailFirstOrder* fo) {
  if (!tower_tail_usable(L2, L3, M, lda) || !oa.wo || !oa.out || (oa.rowsum && oa.pre2)) {
    set_error("tower tail: needs two bf16 layers of N <= 400 (Npad = Kpad = 416) and an output head");
    return RMX_E_INVALID;
  }
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  RMX_HIP(hipFuncSetAttribute((const void*)tower_tail_bf16_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kTLds));
  TailArgs p{};
  p.M = M;
  p.nblk = (M + kTBM - 1) / kTBM;
  p.H = H;
  p.lda = lda;
  p.K2 = L2.K;
  p.W2 = L2.W16;
  p.b2 = L2.b;
  p.W3 = L3.W16;
  p.b3 = L3.b;
  p.oa = oa;
  if (fo) {
    if (fo->F > 40 || fo->F <= 0 || !fo->ids || !fo->w || oa.pre) {
      set_error("tower tail: the fused first order needs 1 <= F <= 40 and no precomputed pre");
      return RMX_E_INVALID;
    }
    p.fo_ids = fo->ids;
    p.fo_w = fo->w;
    p.fo_F = fo->F;
    p.fo_wld = fo->wld > 0 ? fo->wld : 1;
  }
  const int grid = std::min(p.nblk, std::max(ncu, 1));
  hipLaunchKernelGGL(tower_tail_bf16_kernel, dim3(grid), dim3(kTThreads), kTLds, s, p);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
