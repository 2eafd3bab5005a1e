// k_fused_s3.hip -- DeepFM's whole fp32 tower in one persistent row-owner kernel on the split GEMM (gfx950),
// BASELINE.json configs[1].
//
// Layer 1 (gathered rows, first order and FM fused: k_head_s3.hip), layer 2 and layer 3 + the output dot and
// the head (k_tail_s3.hip) of DeepFM (model/encoder/HigherOrderEncoder.scala:34-59: three Linear(. -> 400) +
// ReLU over x = Reshape(B, F k) of the gathered embeddings, ParRecModel.scala:279-306; first order
// bnn/Scatter.scala:17-36; FM SecondOrderEncoder.scala:19-34; head DeepFM.scala:54-80: CAddTable + Sigmoid):
//   h1 = ReLU(x W1^T + b1), h2 = ReLU(h1 W2^T + b2)        both in the wave's registers, never in HBM
//   y  = sum_n ReLU(h2 W3^T + b3)[n] wo[n] + bo;  p = sigmoid((y1 + y2) + y + beta)
// Why: as head + tail, layer 1 wrote h1 (109 MB at B = 65,536) in one burst per round of
// blocks and the tail read it back through its own LDS-DMA ring, in a second launch.  With the operands
// swapped (D = W x^T, k_rowown.hpp), a lane holds outputs n = 16 t + 4 g .. + 3 of its sample -- exactly the
// K values lane group g feeds the next layer's split step (K = 32 c + 16 h + 4 g + q) -- so layer 1's
// accumulators ARE layer 2's B operand after bias + ReLU, as h2 already was for layer 3 in the tail.  The
// only HBM traffic left is the ids, the gathered rows + first-order weights, the L2-resident weight planes
// and p.
//
// Per row block (128 rows, a wave owns 16 of them and all 416 columns), one 3-slot weight ring, one barrier
// per unit (one K step x one column half), unit U + 2's DMAs riding unit U's MFMAs:
//   layer 1: 2 KS units -- (c, half 0) then (c, half 1), the A operand (two fields' gathered rows) split once
//            per K step; ids three steps ahead and rows + first-order weights one step ahead (k_head_s3.hip),
//            running on across row blocks: the next block's first rows land during this block's last steps
//   layer 2: 26 units -- (c, half 0), (c, half 1) for c = 0 .. 12, the A operand h1 tiles 2c, 2c + 1 (from
//            registers; they die after step c, so h1 shrinks while acc2 fills: the peak is h1 + acc2 = 200
//            registers at c = 0)
//   layer 3: 26 units -- half 0's 13 steps, then half 1's, each half folding ReLU(. + b3) . wo into the
//            row's logit (k_tail_s3.hip q_layer3)
// Vector-memory instructions per unit: 9 in a layer-1 half-0 unit (1 id + 2 row + 1 weight DMA + 5 planes),
// 5 in every other unit -- every wait is a compile-time vmcnt.
//
// LDS: the ring (3 x 39,936) + per wave [2 A slots | 4 id slots | 2 weight slots] (8 x 4,864) + b3 | wo | b1
// (4,992) = 163,712 B.  b2 is DMA'd per row block into each wave's A slot that layer 1 no longer needs.
//
// Parity: each layer's products and K order are the head's / tail's, so h1, h2 and the logit's summands
// are the same fp32 values; the FM + first order are encoder_k16_kernel<1>'s arithmetic (bit-identical y1 +
// y2), and the head applies out_finish_kernel's order.  The predictions are therefore bitwise those of
// head + tail (tests/test_fused_s3.py), and held to 1e-5 against the fp64 oracle.
#include "k_rowown.hpp"

namespace rmx {
namespace {
using namespace rowown;

constexpr int kFMaxF = 40;                       // fields (K = 16 F <= 640, 20 K steps)
constexpr int kFA = 2 * 2 * 16 * 64;             // per wave: 2 slots x [2 fields][16 samples][64 B]
constexpr int kFId = 4 * 128;                    // per wave: 4 slots x [2 fields][16] ids
constexpr int kFWr = 2 * 128;                    // per wave: 2 slots x [2 fields][16] first-order weights
constexpr int kFWave = kFA + kFId + kFWr;
constexpr int kFKS2 = 13;                        // K steps of layers 2 and 3 (Kpad 416)
constexpr int kFPrm = 3 * kQN;                   // b3 | wo | b1 in LDS
constexpr size_t kFLds = (size_t)kQSlots * kQUnit + (size_t)kQW * kFWave + sizeof(float) * kFPrm;
static_assert(kFLds <= 160 * 1024, "LDS budget");
static_assert(sizeof(float) * kQN <= 2048, "b2 fits a wave's free A slot (f_b2_dma)");

// weight-fragment prefetch depth (column tiles) of the layer-2 units (2 measured the same, 0.3101-0.3102 vs
// 0.3093-0.3101 ms) and the layer-3 units (2 spilled 7 registers)
#ifndef RMX_FUSED_PF2
#define RMX_FUSED_PF2 1
#endif
#ifndef RMX_FUSED_PF3
#define RMX_FUSED_PF3 1
#endif

// Diagnostic builds only (tools/diag_fused.py; never set in librmx.so): bit 1 s_memtime stamps of block 0's
// waves at the layer boundaries of its first row blocks and at every layer-1 unit of row block 1, s_memrealtime
// at the kernel's start and end (the clock); timing probes with wrong results: bit 2 layer 1's row gathers
// from a fixed (cached) address, bit 4 no row / weight gathers in layer 1 at all
#ifndef RMX_FUSED_DIAG
#define RMX_FUSED_DIAG 0
#endif
#if RMX_FUSED_DIAG & 1
constexpr int kFDiagIt = 4, kFDiagPh = 6;
__device__ unsigned long long g_fused_t[kQW][kFDiagIt][kFDiagPh];  // [wave][row block][phase]
__device__ unsigned long long g_fused_clk[kQW][4];                   // memtime / memrealtime at start, end
__device__ unsigned long long g_fused_u[kQW][2 * kFMaxF];            // row block 1's layer-1 units, at entry
// one lane's vector store (the value and the address depend on the lane: never a scalar-cache store)
__device__ __forceinline__ void f_stamp(unsigned long long* dst, int lane, unsigned long long v) {
  int l = lane;
  asm volatile("" : "+v"(l), "+v"(v));
  if (l == 0) dst[l] = v;
}
#define F_USTAMP(it, u)                                                                                  \
  do {                                                                                                   \
    if (blockIdx.x == 0 && (it) == 1) f_stamp(&g_fused_u[w][u], lane, __builtin_amdgcn_s_memtime());     \
  } while (0)
#define F_STAMP(it, ph)                                                                                  \
  do {                                                                                                   \
    if (blockIdx.x == 0 && (it) < kFDiagIt) f_stamp(&g_fused_t[w][it][ph], lane, __builtin_amdgcn_s_memtime()); \
  } while (0)
#else
#define F_STAMP(it, ph) \
  do {                  \
  } while (0)
#define F_USTAMP(it, u) \
  do {                  \
  } while (0)
#endif

struct FusedS3Args {
  int M, F, KS, NU;       // KS = ceil(F / 2) layer-1 K steps; NU = 2 KS + 52 units per row block
  QRows rows;             // full / half row blocks (k_rowown.hpp)
  const int32_t* ids;     // [M][F]
  const float* table;     // row of id at table + (id << gsh) (16 fp32: k = 16)
  int gsh;
  const float* wtab;      // first-order weight of id at wtab[id << wsh]
  int wsh;
  const bf16_t* W1;       // [KS][3][416][32] split planes (DenseLayer::W3)
  const float* b1;        // [416]
  const bf16_t* W2;       // [13][3][416][32]
  const float* b2;
  const bf16_t* W3;
  const float* b3;
  OutArgs oa;             // wo [416], bo, beta, out
  int prio;
  int dma_split;          // the two wave halves issue their DMAs at different tiles (knob "fused_dma_split")
};

// unit u of a row block -> its weight planes (wave-uniform)
__device__ __forceinline__ const bf16_t* f_unit_src(const FusedS3Args& p, int u) {
  const int l1 = 2 * p.KS;
  int c, half;
  const bf16_t* W;
  if (u < l1) {
    c = u >> 1;
    half = u & 1;
    W = p.W1;
  } else if (u < l1 + 2 * kFKS2) {
    const int v = u - l1;
    c = v >> 1;
    half = v & 1;
    W = p.W2;
  } else {
    const int v = u - l1 - 2 * kFKS2;
    half = v >= kFKS2 ? 1 : 0;
    c = v - half * kFKS2;
    W = p.W3;
  }
  return W + (int64_t)(c * 3 * kQN + half * kQUT * 16) * 32;
}

// the source of unit u + d (d <= 2), wrapping into the next row block's first units (the same weights)
__device__ __forceinline__ const bf16_t* f_ahead(const FusedS3Args& p, int u, int d) {
  const int v = u + d;
  return f_unit_src(p, v < p.NU ? v : v - p.NU);
}

// layer 1's unit (c, half) + 2 = (c + 1, half) of W1, or -- at the last K step -- layer 2's (0, half): W1 / W2
// are held in SGPRs across the loop and selected (f_ahead indexed the kernel arguments by a run-time unit, a
// scalar load whose lgkmcnt(0) wait also drained the unit's first LDS reads)
__device__ __forceinline__ const bf16_t* f_ahead1(const bf16_t* W1, const bf16_t* W2, int c, int KS, int half) {
  const bool l1 = c + 1 < KS;
  const bf16_t* W = l1 ? W1 : W2;
  const int cc = l1 ? c + 1 : 0;
  return W + (int64_t)(cc * 3 * kQN + half * kQUT * 16) * 32;
}

// unit V (a compile-time constant after unrolling) of layers 2 + 3 (V < 52), or V - 52 of the next row block's
// layer 1: a kernel-argument pointer made opaque at its use plus a constant offset -- formed from the
// runtime KS, or hoisted out of the row-block loop, the 52 unit sources spilled (SGPRs into VGPR lanes)
__device__ __forceinline__ const bf16_t* f_src23(const FusedS3Args& p, int V) {
  const bf16_t* W = V < 2 * kFKS2 ? p.W2 : (V < 4 * kFKS2 ? p.W3 : p.W1);
  asm volatile("" : "+s"(W));
  int c, half;
  if (V < 2 * kFKS2) {
    c = V >> 1;
    half = V & 1;
  } else if (V < 4 * kFKS2) {
    half = V - 2 * kFKS2 >= kFKS2 ? 1 : 0;
    c = V - 2 * kFKS2 - half * kFKS2;
  } else {
    c = (V - 4 * kFKS2) >> 1;
    half = (V - 4 * kFKS2) & 1;
  }
  return W + (int64_t)(c * 3 * kQN + half * kQUT * 16) * 32;
}

// ids of K step c of the row block at row0 (nw waves own rows) into id slot `slot` (lanes 0 .. 31: field
// 2c + (L >> 4) of sample L & 15; past M or F, or for a wave without rows: -1)  (k_head_s3.hip h_id_dma)
__device__ __forceinline__ void f_id_dma(const FusedS3Args& p, char* wl, int row0, int nw, int c, int slot, int w,
                                         int lane) {
  int f = lane >> 4, r = lane & 15;
  asm volatile("" : "+v"(f), "+v"(r));
  const int m = row0 + w * 16 + r, fld = 2 * c + f;
  const bool ok = w < nw && m < p.M && fld < p.F;
  const int32_t* src = ok ? p.ids + (int64_t)m * p.F + fld : g_rmx_neg1;
  if (lane < 32)
    lds_dma<4>(src, wl + kFA + slot * 128);
}

// rows (2 DMAs) and first-order weights (lanes 0 .. 31) of the wave's step s, from the ids in id slot s & 3,
// into A slot s & 1 / weight slot s & 1  (k_head_s3.hip h_row_dma)
// part 0 / 1: the row of field 2c / 2c + 1; part 2: the weights; -1: all three
__device__ __forceinline__ void f_row_dma(const FusedS3Args& p, char* wl, int s, int lane, int part = -1) {
  const int* ids = reinterpret_cast<const int*>(wl + kFA + (s & 3) * 128);
  int r = lane >> 2, g = swz_slot(lane >> 2, lane & 3), lw = lane & 31;
  asm volatile("" : "+v"(r), "+v"(g), "+v"(lw));
  const float* zero16 = g_rmx_zero16;
  char* a = wl + (s & 1) * 2048;
  if (part < 0 || part == 0) {
    const int id0 = ids[r];
    lds_dma<16>(id0 >= 0 ? p.table + ((int64_t)id0 << p.gsh) + 4 * g : zero16, a);
  }
  if (part < 0 || part == 1) {
    const int id1 = ids[16 + r];
    lds_dma<16>(id1 >= 0 ? p.table + ((int64_t)id1 << p.gsh) + 4 * g : zero16, a + 1024);
  }
  if (part < 0 || part == 2) {
    const int idw = ids[lw];
    if (lane < 32)
      lds_dma<4>(idw >= 0 ? p.wtab + ((int64_t)idw << p.wsh) : zero16, wl + kFA + kFId + (s & 1) * 128);
  }
}

// The same DMAs from ids already in registers (round 6): step s + 1's three ids (the rows of fields 2c, 2c + 1
// and the weight) are read from their id slot at the start of step s's half-0 unit, beside prep's reads.
// Read at the DMA (f_row_dma inside the MFMA stream), each id needed an s_waitcnt lgkmcnt(0) that also drained
// the B fragments prefetched for the next tiles -- three times per half-0 unit.
struct FRowIds {
  int id0, id1, idw;
};
__device__ __forceinline__ FRowIds f_row_ids(char* wl, int s, int lane) {
  const int* ids = reinterpret_cast<const int*>(wl + kFA + (s & 3) * 128);
  int r = lane >> 2, lw = lane & 31;
  asm volatile("" : "+v"(r), "+v"(lw));
  return FRowIds{ids[r], ids[16 + r], ids[lw]};
}
__device__ __forceinline__ void f_row_dma_ids(const FusedS3Args& p, char* wl, int s, int lane, const FRowIds& q,
                                              int part) {
#if RMX_FUSED_DIAG & 4  // timing probe: no row / weight gathers in layer 1 (results wrong)
  return;
#endif
  int g = swz_slot(lane >> 2, lane & 3);
  asm volatile("" : "+v"(g));
  const float* zero16 = g_rmx_zero16;
  char* a = wl + (s & 1) * 2048;
#if RMX_FUSED_DIAG & 2  // timing probe: every gather reads the lane's own row of the table's first 16 (cached)
  if (part == 0) lds_dma<16>(p.table + ((int64_t)(lane >> 2) << p.gsh) + 4 * g, a);
  if (part == 1) lds_dma<16>(p.table + ((int64_t)(lane >> 2) << p.gsh) + 4 * g, a + 1024);
#else
  if (part == 0) lds_dma<16>(q.id0 >= 0 ? p.table + ((int64_t)q.id0 << p.gsh) + 4 * g : zero16, a);
  if (part == 1) lds_dma<16>(q.id1 >= 0 ? p.table + ((int64_t)q.id1 << p.gsh) + 4 * g : zero16, a + 1024);
#endif
  if (part == 2 && lane < 32)
    lds_dma<4>(q.idw >= 0 ? p.wtab + ((int64_t)q.idw << p.wsh) : zero16, wl + kFA + kFId + (s & 1) * 128);
}

// The biases of layers 1 and 2 come from LDS (round 6).  Read with scalar loads (round 5), the compiler
// reused one SGPR quad for all 25 tiles, so every s_load waited out its own round trip before the next:
// s_memtime stamps (tools/diag_fused.py) put the layer-1 epilogue at 8-14 k cycles per row block and the
// end of layer 2 likewise, ~6 % of the kernel.  b1 sits in the block's LDS beside b3 | wo (staged once per
// launch); b2 has no room there, so each wave DMAs it into its own A slot that layer 1's last step freed
// (slot (s - 1) & 1, untouched until the next row block's first rows land), during layer 2's first unit.
__device__ __forceinline__ void f_b2_dma(const FusedS3Args& p, char* wl, int s, int lane) {
  char* dst = wl + ((s - 1) & 1) * 2048;
  const float* zero16 = g_rmx_zero16;
  int l = lane;
  asm volatile("" : "+v"(l));
  lds_dma<16>(p.b2 + 4 * l, dst);                                  // bytes 0 .. 1023
  lds_dma<16>(l < kQN / 4 - 64 ? p.b2 + 256 + 4 * l : zero16, dst + 1024);  // 1024 .. 1663, then zeros
}

// layer-3 half HF (column tiles 13 HF .. + 12; half 1 computes 12, tile 25 is padding): 13 units, one per
// K step, unrolled so that h2's tiles 2c, 2c + 1 are static registers (k_tail_s3.hip q_layer3)
template <int HF, int DOFF>
__device__ __forceinline__ void f_layer3(const FusedS3Args& p, char* lds, const float* prm, f32x4 (&h2)[kQNT],
                                         int& slot, int w, int lane, int lo, int fb, float& part) {
  const int g = lane >> 4;
  f32x4 acc[kQUT];
#pragma unroll
  for (int t = 0; t < kQUT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < kFKS2; ++c) {
    q_enter<5>();
    bf16x8 ah, am, al;
    split3(h2[2 * c], 2 * c + 1 < kQNT ? h2[2 * c + 1] : z, ah, am, al);
    const int dslot = slot == 0 ? 2 : slot - 1;  // (slot + 2) mod 3
    const char* ub = lds + slot * kQUnit;
    const bf16_t* src = f_src23(p, 2 * kFKS2 + HF * kFKS2 + c + 2);
    if constexpr (HF == 0)
      q_unit<kQUT, 0, kQUT, RMX_FUSED_PF3, kQN, DOFF>(ub, fb, ah, am, al, acc, src, lds, dslot, w, lo);
    else
      q_unit<kQUT - 1, 0, kQUT, RMX_FUSED_PF3, kQN, DOFF>(ub, fb, ah, am, al, acc, src, lds, dslot, w, lo);
    slot = q_next(slot);
  }
  // the output dot over this half's columns: ReLU(acc + b3)[n] * wo[n], n = 16 (13 HF + t) + 4 g + q
  constexpr int NT = HF == 0 ? kQUT : kQNT - kQUT;
  __builtin_amdgcn_sched_barrier(0);
  int g4 = 4 * g;
  asm volatile("" : "+v"(g4));
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n0 = 16 * (kQUT * HF + t) + g4;
    const f32x4 bb = *reinterpret_cast<const f32x4*>(prm + n0);
    const f32x4 wv = *reinterpret_cast<const f32x4*>(prm + kQN + n0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = acc[t][r] + bb[r];
      v = v > 0.f ? v : 0.f;
      part += v * wv[r];
    }
  }
  asm volatile("" : "+v"(part));  // (the dot is done here: sunk past half 1 it kept 13 accumulators alive)
}

__global__ __launch_bounds__(kQThreads, 1) void tower_fused_s3_kernel(FusedS3Args p) {
  extern __shared__ __attribute__((aligned(16))) char fsmem[];
  char* lds = fsmem;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  char* wl = fsmem + kQSlots * kQUnit + w * kFWave;  // this wave's rows / ids / weights
  float* prm = reinterpret_cast<float*>(fsmem + kQSlots * kQUnit + kQW * kFWave);  // b3 | wo | b1
  const int nit = p.rows.nit(blockIdx.x);
  const int KS = p.KS;
  const OutArgs& oa = p.oa;
  // knob "fused_prio" (timing A/B): the second-dispatched half of the waves at priority 1 (MI355X_MICROARCH.md,
  // two waves per SIMD item 4)
  if (p.prio && w >= kQW / 2) __builtin_amdgcn_s_setprio(1);
#if RMX_FUSED_DIAG & 1
  if (blockIdx.x == 0) {
    f_stamp(&g_fused_clk[w][0], lane, __builtin_amdgcn_s_memtime());
    f_stamp(&g_fused_clk[w][1], lane, __builtin_amdgcn_s_memrealtime());
  }
#endif

  for (int i = tid; i < 2 * kQN; i += kQThreads) {
    const int a = i / kQN, n = i - a * kQN;
    const float* src = a == 0 ? p.b3 : oa.wo;
    prm[i] = src ? src[n] : 0.f;
  }
  // (a separate loop: a third source in the select above hit "illegal VGPR to SGPR copy" in the compiler)
  for (int i = tid; i < kQN; i += kQThreads) prm[2 * kQN + i] = p.b1[i];
  int lo = (lane >> 2) * 32 + swz_slot(lane >> 2, lane & 3) * 8;
  asm volatile("" : "+v"(lo));
  const int fb = q_fbase(lane);

  // the wave's layer-1 steps s = 0, 1, ... run over its row blocks: step s is K step s % KS of row block
  // blockIdx.x + (s / KS) gridDim.x; its ring slots are s & 3 (ids) and s & 1 (rows, weights)
  auto id_dma = [&](int s) {
    const int it = s / KS, c = s - it * KS;
    int row0, nw;
    p.rows.desc(blockIdx.x, it, row0, nw);
    f_id_dma(p, wl, row0, nw, c, s & 3, w, lane);
  };
  if (nit > 0) {
    for (int s = 0; s < 3; ++s) id_dma(s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    f_row_dma(p, wl, 0, lane);
#pragma unroll
    for (int qq = 0; qq < kQQ; ++qq) q_dma(f_unit_src(p, 0), lds, 0, w, qq, lo);
#pragma unroll
    for (int qq = 0; qq < kQQ; ++qq) q_dma(f_unit_src(p, 1), lds, 1, w, qq, lo);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // prm staged; this wave's units 0 and 1 landed (q_enter's barrier covers the rest)

  int slot = 0, s = 0;
  // Round 6: the two waves of a SIMD (w and w + 4) issue their DMAs at different tiles of each unit -- the
  // first half at tiles 0 .. 4 (and layer 1's gathers at 6 .. 11), the second half at tiles 6 .. 10 (gathers
  // at 0 .. 3) -- so an LDS-DMA issue that holds one wave for ~100-200 cycles meets the partner's MFMAs
  // instead of the partner's own DMA issue.  The vector-memory instructions per unit are the same, so every
  // static vmcnt holds.  Each half runs its own copy of the loop (LATE is a compile-time flag; knob
  // "fused_dma_split": 1 the second half late; 2 (default since late round 6) every wave late, i.e. layer 1's
  // gathers at the head of each half-0 unit -- half a unit more lead on the row lines: configs[3]'s V = 100M
  // partition +1.3 / +1.9 % on two boxes, V = 1M neutral, profiles/r06/ab_fused_dma2.txt; 0: every wave early).
  const bool late = (w >= kQW / 2 && p.dma_split) || p.dma_split == 2;  // (2: every wave on the late tiles)
  auto body = [&](auto LATE) {
  constexpr bool kLate = decltype(LATE)::value != 0;
  constexpr int kDoff = kLate ? 6 : 0;
  for (int it = 0; it < nit; ++it) {
    int row0, nw;
    p.rows.desc(blockIdx.x, it, row0, nw);
    if (w >= nw) {
      // a half block's waves 4 .. 7: the same units, barriers and DMAs (ids of no rows), no MFMAs -- one
      // branch per row block (per-unit branches spilled the accumulators)
#pragma unroll 1
      for (int c = 0; c < KS; ++c, ++s) {
        q_enter<5>();
        id_dma(s + 3);
        f_row_dma(p, wl, s + 1, lane);
        __builtin_amdgcn_sched_barrier(0);
        int dslot = slot == 0 ? 2 : slot - 1;
        q_dma_only(f_ahead(p, 2 * c, 2), lds, dslot, w, lo);
        slot = q_next(slot);
        q_enter<9>();
        dslot = slot == 0 ? 2 : slot - 1;
        q_dma_only(f_ahead(p, 2 * c + 1, 2), lds, dslot, w, lo);
        slot = q_next(slot);
      }
#pragma unroll 1
      for (int u = 2 * KS; u < p.NU; ++u) {
        q_enter<5>();
        const int dslot = slot == 0 ? 2 : slot - 1;
        q_dma_only(f_ahead(p, u, 2), lds, dslot, w, lo);
        slot = q_next(slot);
      }
      continue;
    }
    // ---- layer 1 (+ first order + FM): units (c, half 0), (c, half 1) ----
    F_STAMP(it, 0);
    f32x4 h1[kQNT];
#pragma unroll
    for (int t = 0; t < kQNT; ++t) h1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 fs = f32x4{0.f, 0.f, 0.f, 0.f}, fq = fs;
    float y1 = 0.f;
    bf16x8 ah, am, al;
    // step ss's A operand from its rows in A slot ss & 1: FM sums + first order (field order) and the split
    auto prep = [&](int ss) {
      int o = r16 * 64 + swz_slot(r16, g) * 16;
      asm volatile("" : "+v"(o));
      const char* a = wl + (ss & 1) * 2048;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(a + o);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(a + 1024 + o);
      const float* wr = reinterpret_cast<const float*>(wl + kFA + kFId + (ss & 1) * 128);
      {
#pragma clang fp contract(off)
        fm_accum(a0, a1, fs, fq);  // (SecondOrderEncoder sums, field order, k_gemm.hpp)
        y1 += wr[r16];             // first order in field order (encoder_k16_kernel<0>)
        y1 += wr[16 + r16];
      }
      split3(a0, a1, ah, am, al);
    };
    const bf16_t* W1 = p.W1;
    const bf16_t* W2 = p.W2;
    asm volatile("" : "+s"(W1), "+s"(W2));  // (loaded once per row block, selected per unit)
    // (forming step s + 1's A at the end of step s's half-1 unit, before the barrier, measured the same:
    // 0.3086-0.3097 vs 0.3094-0.3098 ms, profiles/r05/ab_fused.txt -- not kept)
#pragma unroll 1
    for (int c = 0; c < KS; ++c, ++s) {
      q_enter<5>();  // previous unit: (c - 1, half 1) or the previous row block's last layer-3 unit, 5 DMAs
      F_USTAMP(it, 2 * c);
      // step s + 1's ids landed two steps ago (its id DMA rode step s - 2; every q_enter since waited for it)
      const FRowIds nid = f_row_ids(wl, s + 1, lane);
      prep(s);
      int dslot = slot == 0 ? 2 : slot - 1;
      // the ids (3 steps ahead), rows and weights (1 step ahead) ride tiles 6, 8, 10, 11 of the unit's MFMA
      // stream, after its 5 plane DMAs: an LDS-DMA issue can hold its wave ~100-200 cycles, and four of them
      // ahead of the unit's first MFMA (k_head_s3.hip's order) cost 2 % (0.3142-0.3162 vs 0.3088-0.3111 ms)
      const int sn = s;
      auto extra = [&](int t) {
        if (t == (kLate ? 0 : 6)) id_dma(sn + 3);
        if (t == (kLate ? 1 : 8)) f_row_dma_ids(p, wl, sn + 1, lane, nid, 0);
        if (t == (kLate ? 2 : 10)) f_row_dma_ids(p, wl, sn + 1, lane, nid, 1);
        if (t == (kLate ? 3 : 11)) f_row_dma_ids(p, wl, sn + 1, lane, nid, 2);
      };
      q_unit<kQUT, 0, kQNT, 2, kQN, kDoff>(lds + slot * kQUnit, fb, ah, am, al, h1, f_ahead1(W1, W2, c, KS, 0), lds, dslot, w, lo,
                                          true, extra);
      slot = q_next(slot);
      q_enter<9>();  // previous unit: 1 id + 2 row + 1 weight + 5 plane DMAs
      F_USTAMP(it, 2 * c + 1);
      dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kQNT - kQUT, kQUT, kQNT, 2, kQN, kDoff>(lds + slot * kQUnit, fb, ah, am, al, h1, f_ahead1(W1, W2, c, KS, 1), lds,
                                                    dslot, w, lo);
      slot = q_next(slot);
    }
    __builtin_amdgcn_sched_barrier(0);
    F_STAMP(it, 1);
    // first order + FM of the row (k_head_s3.hip's epilogue: encoder_k16_kernel<1>'s arithmetic)
    float pre;
    {
#pragma clang fp contract(off)
      float a = 0.f;
      float d[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) d[t] = fs[t] * fs[t] - fq[t];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
#pragma unroll
        for (int t = 0; t < 4; ++t) a += __shfl(d[t], gg * 16 + r16);
      pre = y1 + 0.5f * (a / 16.0f);
    }
    asm volatile("" : "+v"(pre));  // (formed here: sunk to the head, its 16 shuffled terms were spilled)
    // h1 = ReLU(acc1 + b1), in place (b1 from LDS)
    {
      int o = 4 * g;
      asm volatile("" : "+v"(o));
#pragma unroll
      for (int t = 0; t < kQNT; ++t) h1[t] = relu4(h1[t] + *reinterpret_cast<const f32x4*>(prm + 2 * kQN + 16 * t + o));
    }
    // ---- layer 2: units (c, half 0), (c, half 1); h1 tiles 2c, 2c + 1 die after step c ----
    F_STAMP(it, 2);
    f32x4 h2[kQNT];
#pragma unroll
    for (int t = 0; t < kQNT; ++t) h2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int sb2 = s;  // (b2 goes to A slot (sb2 - 1) & 1: f_b2_dma)
#pragma unroll
    for (int c = 0; c < kFKS2; ++c) {
      q_enter<5>();
      bf16x8 ah, am, al;
      const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
      split3(h1[2 * c], 2 * c + 1 < kQNT ? h1[2 * c + 1] : z, ah, am, al);
      int dslot = slot == 0 ? 2 : slot - 1;
      // unit (0, half 0) also DMAs b2 into this wave's free A slot, at its last tile (after the 5 plane DMAs)
      auto b2x = [&](int t) {
        if (c == 0 && t == kQUT - 1) f_b2_dma(p, wl, sb2, lane);
      };
      q_unit<kQUT, 0, kQNT, RMX_FUSED_PF2, kQN, kDoff>(lds + slot * kQUnit, fb, ah, am, al, h2, f_src23(p, 2 * c + 2),
                                                       lds, dslot, w, lo, true, b2x);
      slot = q_next(slot);
      if (c == 0)
        q_enter<7>();  // 5 plane DMAs + the 2 of b2
      else
        q_enter<5>();
      dslot = slot == 0 ? 2 : slot - 1;
      q_unit<kQNT - kQUT, kQUT, kQNT, RMX_FUSED_PF2, kQN, kDoff>(lds + slot * kQUnit, fb, ah, am, al, h2, f_src23(p, 2 * c + 3),
                                                     lds, dslot, w, lo);
      slot = q_next(slot);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      // b2 from this wave's A slot (its DMA landed units ago: every later q_enter waited for it)
      // (the lane id made afresh by mbcnt: kept from the kernel's start, lane & 48 was spilled to scratch)
      const int ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
      int o = ((sb2 - 1) & 1) * 2048 + 16 * (ln >> 4);
      asm volatile("" : "+v"(o));
#pragma unroll
      for (int t = 0; t < kQNT; ++t) h2[t] = relu4(h2[t] + *reinterpret_cast<const f32x4*>(wl + o + 64 * t));
    }
    // ---- layer 3 + the output dot ----
    F_STAMP(it, 3);
    float part = 0.f;
    f_layer3<0, kDoff>(p, lds, prm, h2, slot, w, lane, lo, fb, part);
    F_STAMP(it, 4);
    f_layer3<1, kDoff>(p, lds, prm, h2, slot, w, lane, lo, fb, part);
    F_STAMP(it, 5);
    // ---- head: the four lane groups' columns, then bias, CAddTable, sigmoid (out_finish_kernel's order) ----
    part += __shfl_xor(part, 16);
    part += __shfl_xor(part, 32);
    // (lane made afresh, as for b2: the kernel-start r16 was spilled here, and its reload waited vmcnt(0) --
    // for every DMA in flight, the next row block's first units included)
    const int ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const int m = row0 + w * 16 + (ln & 15);
    if (ln < 16 && m < p.M) {
      float y = part;
      if (oa.has_bo) y = y + oa.bo;
      float tt = pre + y;
      tt = tt + oa.beta;
      oa.out[m] = 1.0f / (1.0f + expf(-tt));
    }
  }
  };
  if (late)
    body(std::integral_constant<int, 1>{});
  else
    body(std::integral_constant<int, 0>{});
  // the ring's trailing DMAs (units 0 / 1 of a row block that does not exist, the next block's ids / rows)
  // land before the block's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if RMX_FUSED_DIAG & 1
  if (blockIdx.x == 0) {
    f_stamp(&g_fused_clk[w][2], lane, __builtin_amdgcn_s_memtime());
    f_stamp(&g_fused_clk[w][3], lane, __builtin_amdgcn_s_memrealtime());
  }
#endif
}

}  // namespace

#if RMX_FUSED_DIAG & 1
// out: [8 waves][4 row blocks][6 stamps], [8 waves][4] (memtime, memrealtime at start and end), then
// [8 waves][80] row block 1's layer-1 unit entries
extern "C" int rmx_diag_fused(unsigned long long* out) {
  RMX_HIP(hipDeviceSynchronize());
  RMX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fused_t), sizeof(g_fused_t)));
  RMX_HIP(hipMemcpyFromSymbol(out + sizeof(g_fused_t) / 8, HIP_SYMBOL(g_fused_clk), sizeof(g_fused_clk)));
  RMX_HIP(hipMemcpyFromSymbol(out + (sizeof(g_fused_t) + sizeof(g_fused_clk)) / 8, HIP_SYMBOL(g_fused_u),
                              sizeof(g_fused_u)));
  return RMX_OK;
}
#endif

bool tower_fused_s3_usable(const DenseLayer& L1, const DenseLayer& L2, const DenseLayer& L3, int M, int F, int k,
                           bool ids) {
  if (M <= 0 || !ids || k != 16 || F < 1 || F > kFMaxF || !f32_split_enabled()) return false;
  if (!L1.W3 || !L2.W3 || !L3.W3 || L1.W16 || L2.W16 || L3.W16) return false;
  if (!(L1.K == 16 * F && L1.N == 400 && L1.Npad == kQN && L1.N1 < 0 && L1.bias_mode == 1 && L1.K1 < 0)) return false;
  if (!(L2.K == 400 && L2.N == 400 && L3.K == 400 && L3.N == 400 && L2.Npad == kQN && L3.Npad == kQN &&
        (L2.Kpad + 31) / 32 == kFKS2 && (L3.Kpad + 31) / 32 == kFKS2 && L2.N1 < 0 && L3.N1 < 0 && L2.bias_mode == 1 &&
        L3.bias_mode == 1))
    return false;
  if (!L1.b || !L2.b) return false;
  // knob "s3_fused": 0 off (head + tail), 1 (default) / 2 on.  Round 5 kept it to batches whose full 128-row
  // blocks fill every CU (B = 16,384: head + tail 154.4 M against the fused tower's 147.7 M then,
  // profiles/r05/ab_fused_batch.txt); after round 6's fused-tower work it wins at every batch the small-batch
  // kernels leave to it (they take B <= 8,192 first): B = 9,216 / 12,288 / 16,384 / 24,576 107 / 142 / 173 / 180 M
  // against head + tail's 90 / 119 / 152 / 157 M (profiles/r06/ab_fused_mid_batches.txt)
  return tuning_get("s3_fused", 1) != 0;
}

int launch_tower_fused_s3(hipStream_t s, const DenseLayer& L1, const DenseLayer& L2, const DenseLayer& L3, int M, int F,
                          const int32_t* ids, const float* table, int ld, const float* wtab, int wld,
                          const OutArgs& oa) {
  if (!ids || !oa.wo || !oa.out || F < 1 || F > kFMaxF || !L1.W3 || !L2.W3 || !L3.W3 || !L1.b || !L2.b ||
      L1.K != 16 * F || L1.Npad != kQN || L2.Npad != kQN || L3.Npad != kQN || L2.K != 400 || L3.K != 400 ||
      L1.N != 400 || L2.N != 400 || L3.N != 400) {
    set_error("fp32 fused tower: needs a k = 16 gather (F <= 40, ids) into three 400-wide split-GEMM layers + head");
    return RMX_E_INVALID;
  }
  if (M <= 0) return RMX_OK;
  const int l = ld > 0 ? ld : 16, wl = wld > 0 ? wld : 1;
  if ((l & (l - 1)) || l < 16 || (wl & (wl - 1))) {
    set_error("fp32 fused tower: table / weight strides must be powers of two");
    return RMX_E_INVALID;
  }
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  RMX_HIP(hipFuncSetAttribute((const void*)tower_fused_s3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kFLds));
  FusedS3Args p{};
  p.M = M;
  int grid = 0;
  p.rows = q_rows(M, ncu, grid);
  p.F = F;
  p.KS = (F + 1) / 2;
  p.NU = 2 * p.KS + 4 * kFKS2;
  p.ids = ids;
  p.table = table;
  p.gsh = __builtin_ctz((unsigned)l);
  p.wtab = wtab;
  p.wsh = __builtin_ctz((unsigned)wl);
  p.W1 = L1.W3;
  p.b1 = L1.b;
  p.W2 = L2.W3;
  p.b2 = L2.b;
  p.W3 = L3.W3;
  p.b3 = L3.b;
  p.oa = oa;
  p.prio = tuning_get("fused_prio", 0);
  p.dma_split = tuning_get("fused_dma_split", 2);
  hipLaunchKernelGGL(tower_fused_s3_kernel, dim3(grid), dim3(kQThreads), kFLds, s, p);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
