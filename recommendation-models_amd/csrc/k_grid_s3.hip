// k_grid_s3.hip -- DeepFM's whole fp32 tower for small launch batches as a 2-D grid of row groups x column
// groups in one cooperative launch, on the split GEMM (gfx950).  BASELINE.json configs[1] at SURVEY.md §8's
// default launch batch (B = 4,096) and the reference's own small batches (DeepFMLocalExample.scala:16).
//
// The tower (model/encoder/HigherOrderEncoder.scala:34-59: Linear(F k -> 400) + ReLU, 400 -> 400 + ReLU,
// 400 -> 400 + ReLU, Linear(400 -> 1)), the first order (bnn/Scatter.scala:17-36), the FM second order
// (SecondOrderEncoder.scala:19-34) and DeepFM's head (DeepFM.scala:54-80: CAddTable + Sigmoid).
//
// Why.  Below ~16 K samples a kernel that gives each block a set of rows and ALL columns
// (k_small_s3.hip: 16-sample blocks; k_fused_s3.hip: 128-row blocks) makes every CU stream the whole tower's
// split weights (3.67 MB) however few rows it owns, at the ~70 GB/s per CU that all 256 CUs streaming from
// L2 / the Infinity Cache get: ~52 us per block, 65 M examples/s at B = 4,096.  Here block (r, c) owns row
// group r (128 rows: a wave owns 16) and column group c (NT of the 25 column tiles of every layer), so it
// streams only NT / 25 of the weights and its rows' inputs: per CU ~0.5 MB of weights + ~0.75 MB of
// activations at B = 4,096 (NT = 4, 7 column groups x 32 row groups = 224 blocks).  Layer l + 1 needs all
// columns of layer l for its rows, so the C blocks of a row group hand their activations over through
// global memory inside the launch (cdna_hip_programming.md §6 Guideline 16): payload stored sc1
// (write-through) and drained by every storing wave, a workgroup barrier, one agent-scope atomic add on the
// row group's counter; the consumer polls the counter relaxed (one lane, bounded, s_sleep), ONE agent-scope
// acquire, then plain loads.  Counters are zeroed by a memset node before every launch; the launch is
// cooperative (every block resident, or the launch fails instead of hanging).  The last hand-off carries
// the C partial logits of each row to column group 0, which sums them in column-group order and applies
// the head.
//
// Per block, the k_rowown.hpp machinery with NT-tile units: a unit = one K step of the block's NT column
// tiles (3 NT pieces of 1 KiB: the three split planes of each tile), a 3-slot LDS-DMA ring, one barrier per
// unit, unit U + 2's pieces issued during unit U; swapped MFMAs (D = W x^T): lane (r16, g) holds outputs
// 16 T + 4 g .. + 3 of its row, which it stores to h[m][16 T + 4 g] as one 16-B sc1 store.  A operands:
// layer 1 gathers its two fields' 64-B rows per K step (ids 4 steps ahead, rows + first-order weights 2
// steps ahead, per-wave LDS slots, as k_fused_s3.hip); layers 2 / 3 stream their 16 rows x 32 K of h (2 steps
// ahead).  Vector-memory instructions per unit per wave are static (layer 1: 4 + Q; layers 2 / 3: 2 + Q), so
// every wait is a compile-time vmcnt.
//
// Arithmetic: each output's products and K order are the split engine's (the six bf16 products per K step,
// smallest first), the FM + first order encoder_k16_kernel<1>'s (bit-identical), so h1 and h2 are the fused
// tower's values bit for bit; only the logit's summation order differs (per column group, then across the
// groups in order): tests/test_grid_s3.py holds it to 5e-6 against the fused / head + tail towers and 1e-5
// against the fp64 oracle.
#include "k_rowown.hpp"

namespace rmx {
namespace {
using namespace rowown;

constexpr int kGW = 8;                   // waves per block
constexpr int kGThreads = kGW * 64;
constexpr int kGRows = kGW * 16;         // rows per row group
constexpr int kGMaxF = 40;
constexpr int kGKS2 = 13;                // K steps of layers 2 / 3

// NT column tiles per block; L units of lead: the weight ring, the A slots (per wave: 2 KiB each -- two fields'
// rows of 16 samples, or 16 rows x 32 K of h), the first-order weight slots and the id slots all hold L + 1
// units.  A unit of a few tiles lasts well under the L2 / Infinity-Cache latency, so the ring has to run
// several units ahead (Little's law: in-flight bytes / latency = the CU's fetch rate); L is as deep as LDS
// allows for the NT (the A slots dominate: 16 KiB per unit per block).
template <int NT, int L>
struct GCfg {
  static constexpr int S = L + 1;                   // slots of every ring
  static constexpr int NINS = 3 * NT;              // 1-KiB pieces per unit
  static constexpr int Q = (NINS + kGW - 1) / kGW;  // per wave (the last wave repeats a piece when short)
  static constexpr int UNIT = NINS * 1024;
  static constexpr int A = S * 2048, ID = S * 128, WR = S * 128;
  static constexpr int WAVE = A + ID + WR;          // per-wave LDS
  static constexpr int PRM = 4 * 16 * NT;          // b1 | b2 | b3 | wo of the block's columns
  static constexpr size_t LDS = (size_t)S * UNIT + (size_t)kGW * WAVE + sizeof(float) * PRM + 16;
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

struct GridArgs {
  int M, F, KS1, R, C;
  const int32_t* ids;     // [M][F]
  const float* table;     // row of id at table + (id << gsh)
  int gsh;
  const float* wtab;      // first-order weight of id at wtab[id << wsh]
  int wsh;
  const bf16_t* W[3];     // split planes [KS_l][3][416][32]
  const float* b[3];      // [416]
  OutArgs oa;             // wo [416], bo, beta, out
  float* h1;              // [M][416] scratch: layer 1's output (hand-off)
  float* h2;              // [M][416] layer 2's output
  float* part;            // [C][M] partial logits
  uint32_t* cnt;          // [R] hand-off counters (zeroed before the launch)
  uint32_t* tmo;          // timeout word (zeroed before the launch; set when a spin gives up)
};

__device__ __forceinline__ int g_clamp_tile(int T) { return T < kQNT ? T : kQNT; }  // tile 25: zero weights

// piece q of this wave in unit (layer of W, K step c) of column group cg into ring slot `slot`
template <int NT, int L>
__device__ __forceinline__ void g_wdma(const bf16_t* W, int c, int cg, char* lds, int slot, int w, int q, int lo) {
  using Cfg = GCfg<NT, L>;
  int ins = w + q * kGW;
  ins = ins < Cfg::NINS ? ins : Cfg::NINS - 1;
  const int pl = ins / NT, tl = ins - pl * NT;
  const int T = g_clamp_tile(cg * NT + tl);
  int l = lo;
  asm volatile("" : "+v"(l));
  const bf16_t* s = W + ((int64_t)(c * 3 + pl) * kQN + 16 * T) * 32 + l;
  lds_dma<16>(s, lds + slot * Cfg::UNIT + ins * 1024);
}

// the weight source (layer, K step) of unit u of the launch's unit sequence (layer 1: KS1 units, then 13 +
// 13); past the end: the last unit again (the trailing DMAs of a ring that runs L units ahead)
__device__ __forceinline__ void g_unit_of(const GridArgs& p, int u, const bf16_t*& W, int& c) {
  const int n = p.KS1 + 2 * kGKS2;
  u = u < n ? u : n - 1;
  if (u < p.KS1) {
    W = p.W[0];
    c = u;
  } else if (u < p.KS1 + kGKS2) {
    W = p.W[1];
    c = u - p.KS1;
  } else {
    W = p.W[2];
    c = u - p.KS1 - kGKS2;
  }
}

// one unit's MFMAs over the block's NT tiles, unit U + L's Q pieces riding tiles 0 .. Q - 1
template <int NT, int L>
__device__ __forceinline__ void g_unit(const char* ub, int fb, const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                       f32x4 (&acc)[NT], const bf16_t* dW, int dc, int cg, char* lds, int dslot, int w,
                                       int lo) {
  constexpr int PF = NT >= 2 ? 2 : 1;
  static_assert(GCfg<NT, L>::Q <= NT, "the unit's DMAs ride its tiles");
  f32x4 bq[PF + 1][3];
  int fbu = fb;
  asm volatile("" : "+v"(fbu));
  auto ldb = [&](int t, f32x4* b) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) b[pl] = *reinterpret_cast<const f32x4*>(ub + fbu + (pl * NT + t) * 1024);
  };
#pragma unroll
  for (int t = 0; t < PF && t < NT; ++t) ldb(t, bq[t]);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t + PF < NT) ldb(t + PF, bq[(t + PF) % (PF + 1)]);
    if (t < GCfg<NT, L>::Q) g_wdma<NT, L>(dW, dc, cg, lds, dslot, w, t, lo);
    __builtin_amdgcn_sched_barrier(0);
    const f32x4* b = bq[t % (PF + 1)];
    const bf16x8 bh = __builtin_bit_cast(bf16x8, b[0]);
    const bf16x8 bm = __builtin_bit_cast(bf16x8, b[1]);
    const bf16x8 bl = __builtin_bit_cast(bf16x8, b[2]);
    f32x4 d = acc[t];
    // the engine's product order (k_gemm.hpp compute_step_s3), operands swapped: smallest terms first
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, am, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, am, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, ah, d, 0, 0, 0);
    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, d, 0, 0, 0);
  }
}

// ids of K step c (lanes 0 .. 31: field 2c + (L >> 4) of the wave's row L & 15; -1 past M / F / the last step)
// into id slot c % S
template <int NT, int L>
__device__ __forceinline__ void g_id_dma(const GridArgs& p, char* wl, int row0, int c, int w, int lane) {
  using Cfg = GCfg<NT, L>;
  int f = lane >> 4, r = lane & 15;
  asm volatile("" : "+v"(f), "+v"(r));
  const int m = row0 + w * 16 + r, fld = 2 * c + f;
  const bool ok = m < p.M && fld < p.F && c < p.KS1;
  const int32_t* src = ok ? p.ids + (int64_t)m * p.F + fld : g_rmx_neg1;
  if (lane < 32) lds_dma<4>(src, wl + Cfg::A + (c % Cfg::S) * 128);
}

// rows (2 DMAs) and first-order weights of K step c from its ids (id slot c % S) into A slot c % S / weight slot
template <int NT, int L>
__device__ __forceinline__ void g_row_dma(const GridArgs& p, char* wl, int c, int lane) {
  using Cfg = GCfg<NT, L>;
  const int sl = c % Cfg::S;
  const int* ids = reinterpret_cast<const int*>(wl + Cfg::A + sl * 128);
  int r = lane >> 2, g = swz_slot(lane >> 2, lane & 3), lw = lane & 31;
  asm volatile("" : "+v"(r), "+v"(g), "+v"(lw));
  const int id0 = ids[r], id1 = ids[16 + r], idw = ids[lw];
  const float* zero16 = g_rmx_zero16;
  char* a = wl + sl * 2048;
  lds_dma<16>(id0 >= 0 ? p.table + ((int64_t)id0 << p.gsh) + 4 * g : zero16, a);
  lds_dma<16>(id1 >= 0 ? p.table + ((int64_t)id1 << p.gsh) + 4 * g : zero16, a + 1024);
  if (lane < 32) lds_dma<4>(idw >= 0 ? p.wtab + ((int64_t)idw << p.wsh) : zero16, wl + Cfg::A + Cfg::ID + sl * 128);
}

// 16 rows x 32 K of h (K step c, columns 32 c ..) into A slot c % S (k_tail_s3.hip q_h1_dma: lane L, instruction
// i: row 8 i + (L >> 3), physical 16-B slot L & 7 = logical slot (L & 7) ^ (row & 7)); past M or past the last
// step: the zero row
template <int NT, int L>
__device__ __forceinline__ void g_h_dma(const GridArgs& p, const float* H, char* wl, int row0, int c, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int r = 8 * i + (lane >> 3), j = (lane & 7) ^ ((lane >> 3) & 7);
    asm volatile("" : "+v"(r), "+v"(j));
    const int m = row0 + w * 16 + r;
    const bool ok = m < p.M && c < kGKS2;
    const float* src = ok ? H + (int64_t)m * kQN + 32 * c + 4 * j : g_rmx_zero16;
    lds_dma<16>(src, wl + (c % GCfg<NT, L>::S) * 2048 + i * 1024);
  }
}

// the h fragment of step c from its slot (zero at step 12's upper half: columns 400 .. 415 are padding)
template <int NT, int L>
__device__ __forceinline__ void g_h_read(const char* wl, int c, int lane, f32x4& a0, f32x4& a1) {
  const int r = lane & 15, g = lane >> 4;
  int o0 = r * 128 + ((g ^ (r & 7)) << 4), o1 = r * 128 + (((g + 4) ^ (r & 7)) << 4);
  asm volatile("" : "+v"(o0), "+v"(o1));
  const char* h = wl + (c % GCfg<NT, L>::S) * 2048;
  a0 = *reinterpret_cast<const f32x4*>(h + o0);
  a1 = *reinterpret_cast<const f32x4*>(h + o1);
  if (c == kGKS2 - 1) a1 = f32x4{0.f, 0.f, 0.f, 0.f};
}

// 16-B write-through store (Guideline 16 R1: the hand-off payload)
__device__ __forceinline__ void g_store_sc1(float* p, const f32x4& v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void g_store1_sc1(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

// publish: every storing wave drains its sc1 stores, the workgroup meets, one lane adds to the counter
__device__ __forceinline__ void g_publish(uint32_t* cnt, int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// consume: one lane polls the counter (relaxed, bounded), ONE agent-scope acquire, the workgroup meets.
// false: the spin gave up (the timeout word is set; the caller writes NaN outputs).  ok_s: an LDS word
__device__ __forceinline__ bool g_acquire(uint32_t* cnt, uint32_t want, uint32_t* tmo, int tid, int& ok_s) {
  if (tid == 0) {
    int ok = 1;
    for (uint32_t spins = 0;; ++spins) {
      if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) break;
      if (spins > (1u << 20) || __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok_s = ok;
  }
  __syncthreads();
  return ok_s != 0;
}

template <int NT, int L>
__global__ __launch_bounds__(kGThreads, 1) void tower_grid_s3_kernel(GridArgs p) {
  extern __shared__ __attribute__((aligned(16))) char gsmem[];
  using Cfg = GCfg<NT, L>;
  constexpr int S = Cfg::S;
  char* lds = gsmem;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  char* wl = gsmem + S * Cfg::UNIT + w * Cfg::WAVE;
  float* prm = reinterpret_cast<float*>(gsmem + S * Cfg::UNIT + kGW * Cfg::WAVE);  // [4][16 NT]
  int& ok_s = *reinterpret_cast<int*>(prm + Cfg::PRM);
  const int r = blockIdx.x / p.C, cg = blockIdx.x - r * p.C;
  const int row0 = r * kGRows;
  const int KS1 = p.KS1;
  const int m = row0 + w * 16 + r16;  // this lane's row
  uint32_t* cnt = p.cnt + r;

  for (int i = tid; i < 4 * 16 * NT; i += kGThreads) {
    const int a = i / (16 * NT), n = cg * NT * 16 + (i - a * 16 * NT);
    const float* src = a == 0 ? p.b[0] : (a == 1 ? p.b[1] : (a == 2 ? p.b[2] : p.oa.wo));
    prm[i] = (src && n < 400) ? src[n] : 0.f;
  }
  int lo = (lane >> 2) * 32 + swz_slot(lane >> 2, lane & 3) * 8;
  asm volatile("" : "+v"(lo));
  const int fb = q_fbase(lane);

  // prologue: ids of steps 0 .. L, rows of steps 0 .. L - 1 (reading those ids), then the ids of steps L + 1 ..
  // 2L - 1 into the slots of steps 0 .. L - 2 (their ids already read), the weights of units 0 .. L - 1
  for (int c = 0; c <= L; ++c) g_id_dma<NT, L>(p, wl, row0, c, w, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int c = 0; c < L; ++c) g_row_dma<NT, L>(p, wl, c, lane);
  for (int c = L + 1; c < 2 * L; ++c) g_id_dma<NT, L>(p, wl, row0, c, w, lane);
  {
    const bf16_t* W;
    int c;
    for (int u = 0; u < L; ++u) {
      g_unit_of(p, u, W, c);
#pragma unroll
      for (int q = 0; q < Cfg::Q; ++q) g_wdma<NT, L>(W, c, cg, lds, u, w, q, lo);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int slot = 0, u = 0;
  f32x4 acc[NT];
  // ---- layer 1 (+ first order + FM in column group 0) ----
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 fs = f32x4{0.f, 0.f, 0.f, 0.f}, fq = fs;
  float y1 = 0.f;
#pragma unroll 1
  for (int c = 0; c < KS1; ++c, ++u) {
    // the DMAs of unit c - L (step c's rows, unit c's weights) have landed: only the L - 1 units since may
    // still be in flight (4 + Q vector-memory instructions each)
    q_enter<(L - 1) * (4 + Cfg::Q)>();
    bf16x8 ah, am, al;
    {
      int o = r16 * 64 + swz_slot(r16, g) * 16;
      asm volatile("" : "+v"(o));
      const char* a = wl + (c % S) * 2048;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(a + o);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(a + 1024 + o);
      if (cg == 0) {
#pragma clang fp contract(off)
        const float* wr = reinterpret_cast<const float*>(wl + Cfg::A + Cfg::ID + (c % S) * 128);
        fm_accum(a0, a1, fs, fq);  // (SecondOrderEncoder sums, field order)
        y1 += wr[r16];             // first order in field order (encoder_k16_kernel<0>)
        y1 += wr[16 + r16];
      }
      split3(a0, a1, ah, am, al);
    }
    // ids 2L steps ahead (their slot held step c + L - 1's, read by this wave's row DMA one unit ago), rows +
    // weights L steps ahead (their slots held step c - 1's, read one unit ago)
    g_id_dma<NT, L>(p, wl, row0, c + 2 * L, w, lane);
    g_row_dma<NT, L>(p, wl, c + L, lane);
    __builtin_amdgcn_sched_barrier(0);
    const bf16_t* dW;
    int dc;
    g_unit_of(p, u + L, dW, dc);
    const int dslot = slot == 0 ? S - 1 : slot - 1;  // (slot + L) mod S: unit u - 1's, read before this barrier
    g_unit<NT, L>(lds + slot * Cfg::UNIT, fb, ah, am, al, acc, dW, dc, cg, lds, dslot, w, lo);
    slot = slot == S - 1 ? 0 : slot + 1;
  }
  __builtin_amdgcn_sched_barrier(0);
  float pre = 0.f;
  if (cg == 0) {
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
  // h_l = ReLU(acc + b_l) -> global (sc1), then the hand-off
  auto store_h = [&](float* H, const float* bl) {
    if (m < p.M) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int T = cg * NT + t;
        if (T < kQNT) {
          const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 16 * t + 4 * g);
          g_store_sc1(H + (int64_t)m * kQN + 16 * T + 4 * g, relu4(acc[t] + bb));
        }
      }
    }
  };
  store_h(p.h1, prm);
  g_publish(cnt, tid);
  bool ok = g_acquire(cnt, (uint32_t)p.C, p.tmo, tid, ok_s);

  // ---- layers 2 and 3 ----
#pragma unroll 1
  for (int l = 1; l < 3; ++l) {
    const float* Hin = l == 1 ? p.h1 : p.h2;
    for (int c = 0; c < L; ++c) g_h_dma<NT, L>(p, Hin, wl, row0, c, w, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int c = 0; c < kGKS2; ++c, ++u) {
      q_enter<(L - 1) * (2 + Cfg::Q)>();
      bf16x8 ah, am, al;
      {
        f32x4 a0, a1;
        g_h_read<NT, L>(wl, c, lane, a0, a1);
        split3(a0, a1, ah, am, al);
      }
      g_h_dma<NT, L>(p, Hin, wl, row0, c + L, w, lane);
      __builtin_amdgcn_sched_barrier(0);
      const bf16_t* dW;
      int dc;
      g_unit_of(p, u + L, dW, dc);
      const int dslot = slot == 0 ? S - 1 : slot - 1;
      g_unit<NT, L>(lds + slot * Cfg::UNIT, fb, ah, am, al, acc, dW, dc, cg, lds, dslot, w, lo);
      slot = slot == S - 1 ? 0 : slot + 1;
    }
    __builtin_amdgcn_sched_barrier(0);
    if (l == 1) {
      store_h(p.h2, prm + 16 * NT);
      g_publish(cnt, tid);
      ok = g_acquire(cnt, 2u * p.C, p.tmo, tid, ok_s) && ok;
    }
  }
  // ---- the output dot over the block's columns: ReLU(acc + b3) . wo, then the C groups' partials ----
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const f32x4 bb = *reinterpret_cast<const f32x4*>(prm + 2 * 16 * NT + 16 * t + 4 * g);
    const f32x4 wv = *reinterpret_cast<const f32x4*>(prm + 3 * 16 * NT + 16 * t + 4 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = acc[t][q] + bb[q];
      v = v > 0.f ? v : 0.f;
      part += v * wv[q];
    }
  }
  part += __shfl_xor(part, 16);
  part += __shfl_xor(part, 32);
  if (g == 0 && m < p.M) g_store1_sc1(p.part + (int64_t)cg * p.M + m, part);
  g_publish(cnt, tid);  // (its vmcnt(0) also lands the ring's trailing DMAs before the LDS is released)
  if (cg != 0) return;
  ok = g_acquire(cnt, 3u * p.C, p.tmo, tid, ok_s) && ok;
  // ---- head (column group 0): the partial logits in column-group order, bias, CAddTable, sigmoid ----
  if (g == 0 && m < p.M) {
    float y = 0.f;
    for (int q = 0; q < p.C; ++q) y += p.part[(int64_t)q * p.M + m];
    const OutArgs& oa = p.oa;
    if (oa.has_bo) y = y + oa.bo;
    float tt = pre + y;
    tt = tt + oa.beta;
    oa.out[m] = ok ? 1.0f / (1.0f + expf(-tt)) : __builtin_nanf("");
  }
}

// the lead per column-tile count (as deep as LDS allows: GCfg::LDS <= 160 KiB)
template <int NT>
constexpr int grid_lead() {
  return NT == 1 ? 6 : (NT == 2 ? 5 : (NT == 4 ? 4 : 3));
}

// NT (column tiles per block) for M rows on ncu CUs: the smallest of 1, 2, 4, 7 whose grid (row groups x
// ceil(25 / NT) column groups) fits the CUs -- 0 when none does
int grid_nt(int M, int ncu) {
  const int R = (M + kGRows - 1) / kGRows;
  for (int nt : {1, 2, 4, 7})
    if ((int64_t)R * ((kQNT + nt - 1) / nt) <= ncu) return nt;
  return 0;
}

}  // namespace

bool tower_grid_s3_usable(const rmx_model& m, int M, int F, int k, bool ids) {
  if (M <= 0 || !ids || k != 16 || F < 1 || F > kGMaxF || m.type != RMX_MODEL_DEEPFM || m.layers.size() != 3 ||
      !f32_split_enabled() || m.precision != kF32)
    return false;
  for (int l = 0; l < 3; ++l) {
    const DenseLayer& L = m.layers[l];
    if (!L.W3 || L.W16 || L.N != 400 || L.Npad != kQN || L.N1 >= 0 || L.bias_mode != 1 || L.K1 >= 0 || !L.b) return false;
    if (L.K != (l == 0 ? 16 * F : 400)) return false;
  }
  // knob "s3_grid": 0 off, 1 (default) from M >= s3_grid_min (default 1,024) while a grid fits the CUs, 2 always
  // (while it fits)
  const int knob = tuning_get("s3_grid", 1);
  if (knob == 0) return false;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  if (grid_nt(M, ncu) == 0) return false;
  return knob == 2 || M >= tuning_get("s3_grid_min", 1024);
}

int launch_tower_grid_s3(hipStream_t s, const rmx_model& m, int M, int F, const int32_t* ids, const float* table,
                         int ld, const float* wtab, int wld, const OutArgs& oa, float* h1, float* h2, float* part,
                         uint32_t* sync, size_t sync_bytes) {
  if (M <= 0) return RMX_OK;
  const int l = ld > 0 ? ld : 16, wl = wld > 0 ? wld : 1;
  if ((l & (l - 1)) || l < 16 || (wl & (wl - 1)) || !oa.wo || !oa.out || !h1 || !h2 || !part || !sync) {
    set_error("fp32 grid tower: table / weight strides must be powers of two, an output head and the hand-off buffers");
    return RMX_E_INVALID;
  }
  int dev = 0, ncu = 0;
  RMX_HIP(hipGetDevice(&dev));
  RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  int nt = tuning_get("s3_grid_nt", 0);
  if (nt != 1 && nt != 2 && nt != 4 && nt != 7) nt = grid_nt(M, ncu);
  GridArgs p{};
  p.M = M;
  p.F = F;
  p.KS1 = (F + 1) / 2;
  p.R = (M + kGRows - 1) / kGRows;
  p.C = (kQNT + nt - 1) / nt;
  if (nt == 0 || (int64_t)p.R * p.C > ncu || (size_t)(p.R + 4) * sizeof(uint32_t) > sync_bytes) {
    set_error("fp32 grid tower: the grid does not fit the CUs");
    return RMX_E_INVALID;
  }
  p.ids = ids;
  p.table = table;
  p.gsh = __builtin_ctz((unsigned)l);
  p.wtab = wtab;
  p.wsh = __builtin_ctz((unsigned)wl);
  for (int i = 0; i < 3; ++i) {
    p.W[i] = m.layers[i].W3;
    p.b[i] = m.layers[i].b;
  }
  p.oa = oa;
  p.h1 = h1;
  p.h2 = h2;
  p.part = part;
  p.tmo = sync;          // word 0: timeout; words 4 ..: the row groups' counters (16-B aligned block)
  p.cnt = sync + 4;
  // re-initialise every call (Guideline 16): the polled words, one 16-B-multiple block from the allocation start
  RMX_HIP(hipMemsetAsync(sync, 0, ((p.R + 4) * sizeof(uint32_t) + 15) / 16 * 16, s));
  void* args[] = {&p};
  const dim3 grid(p.R * p.C), block(kGThreads);
  switch (nt) {
#define RMX_GRID_LAUNCH(N)                                                                                         \
  case N: {                                                                                                        \
    constexpr int LL = grid_lead<N>();                                                                             \
    const void* fn = (const void*)tower_grid_s3_kernel<N, LL>;                                                     \
    RMX_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GCfg<N, LL>::LDS));          \
    RMX_HIP(hipLaunchCooperativeKernel(fn, grid, block, args, GCfg<N, LL>::LDS, s));                               \
    break;                                                                                                         \
  }
    RMX_GRID_LAUNCH(1)
    RMX_GRID_LAUNCH(2)
    RMX_GRID_LAUNCH(4)
    RMX_GRID_LAUNCH(7)
#undef RMX_GRID_LAUNCH
    default:
      set_error("fp32 grid tower: bad column-tile count");
      return RMX_E_INVALID;
  }
  return RMX_OK;
}

}  // namespace rmx
