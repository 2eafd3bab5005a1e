// k_gemm.hpp -- the MFMA GEMM engine (fp32, and bf16 for the tower) behind the tower layers and the xDeepFM CIN (gfx950).
//
// Tower layer: BigDL Linear + ReLU chain, model/encoder/HigherOrderEncoder.scala:34-59
// (Linear(in->out, W: out x in, y = b + x W^T) + ReLU per fcDim, then Linear(->1)) and the
// output heads of DeepFM.scala:130-134 / XDeepFM / DCN / PNN (CAddTable + Sigmoid).
// CIN layer: model/xdeepfm/CINEncoder.scala:36-58, 105-176 (+ SURVEY.md Appendix A for L > 1):
//   x0[b,j,f] = e[b,f,j]; z[f*Hp + h] = x0[b,j,f] * u_{l-1}[b,j,h]  (MM(transB = true), :152)
//   u_l[b,j,:] = ReLU(c_l + C_l z)                                   (Linear + ReLU, :154-155)
// a GEMM with M = B*k rows (b, j), K = F * Hp, N = H whose A operand is generated in registers
// (the reference materialises z: B*k x F*Hp floats, 2 GB per layer at B = 4096), and whose
// epilogue folds the output Linear in: rowdot[b*k + j] (+)= sum_h u_l[b,j,h] * W_out[slice_l + h]
// (sum_j sum_h == sum_h sum_j: the pooled pi_l . W_out, :159-176).
//
// All on v_mfma_f32_16x16x4_f32 (exact f32 FMA chain, 64 FLOP/clk/SIMD = the chip's fp32 peak).
// Block = WM waves stacked on M; a wave owns MT*16 rows x all NT*16 columns of the block
// (MT*NT accumulator tiles).  WM is a multiple of 4, so every SIMD carries the same number of
// waves and the one barrier per K stage never waits on an overloaded SIMD.  K is consumed in
// 16-wide chunks; inside a chunk lane group g = lane>>4 owns k = 4g..4g+3, so one ds_read_b128
// per fragment feeds the 4 k-steps of the chunk.  LDS tiles are [rows][16] fp32 with a slot
// XOR-swizzle that keeps the 16-row fragment reads conflict-free for all four ds_read_b128 lane
// groups.  A stage holds BKC chunks; the next stage's global loads are issued before the MFMAs
// of the current one and written to the idle LDS buffer after them (one barrier per stage).
// A operand producers:
//   kDenseA     activations of the previous layer, staged through LDS;
//   kGatherK16  / kGatherAny: first layer, rows gathered straight from the embedding table
//               (ids staged in LDS; x = Reshape(B, F*k) is never materialised);
//   kCinOuter   CIN: a = x0[row][f] * u[row][h-chunk], computed in registers (x0 tile in LDS,
//               u chunk in registers), only the weights go through LDS.
#pragma once

#include <algorithm>
#include <type_traits>

#include "rmx_models.hpp"

namespace rmx {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// physical 16-B slot of logical slot g in row `row` of a [rows][16] fp32 LDS tile
__device__ __forceinline__ int swz_slot(int row, int g) { return g ^ ((4 - ((row >> 2) & 3)) & 3); }

// 16 zero bytes: the LDS-DMA source of out-of-range rows / K padding (a DMA always writes its slot)
static __device__ __attribute__((aligned(16))) float g_rmx_zero16[4];
// id -1 (a zero row): the LDS-DMA source of out-of-range entries of the id ring
static __device__ __attribute__((aligned(16))) int g_rmx_neg1[4] = {-1, -1, -1, -1};


// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be a constant)
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
#define RMX_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    RMX_VMW(0) RMX_VMW(1) RMX_VMW(2) RMX_VMW(3) RMX_VMW(4) RMX_VMW(5) RMX_VMW(6) RMX_VMW(7)
    RMX_VMW(8) RMX_VMW(9) RMX_VMW(10) RMX_VMW(11) RMX_VMW(12) RMX_VMW(13) RMX_VMW(14) RMX_VMW(15)
#undef RMX_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Diagnostic builds only (tools/diag_build.sh; never set in librmx.so): 1 = no A split,
// 2 = no per-step barrier, 4 = no MFMAs in the split GEMM, 32 = no epilogue global stores of the
// activations, 512 = no stored-activation epilogue at all (no LDS transpose either).  Results are
// wrong; timings isolate costs.
#ifndef RMX_GEMM_DIAG
#define RMX_GEMM_DIAG 0
#endif

#if RMX_GEMM_DIAG & 8
// per-phase cycle sums of one wave (block 0, wave 0) of the last split-GEMM launch (tools/diag_phases.py)
// [0, 16): waves 0 and NW/2 of block 0; [16], [17]: s_memtime and s_memrealtime (100 MHz) spans of wave 0
__device__ unsigned long long g_rmx_diag_t[18];
#if RMX_GEMM_DIAG & 256
// per-block timeline of the last selected launch: s_memrealtime at entry / exit, __smid() | XCC id << 16
__device__ unsigned long long g_rmx_blk[4096][3];
#endif
#define RMX_TMARK(k)                                                             \
  do {                                                                           \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                  \
    if (dmark) dsum[k] += _t - dlast;                                            \
    dlast = _t;                                                                  \
  } while (0)
#else
#define RMX_TMARK(k) \
  do {               \
  } while (0)
#endif

#ifndef RMX_STAG_PF
#define RMX_STAG_PF 2
#endif
#ifndef RMX_DIAG_NOB
#define RMX_DIAG_NOB 0  // timing probe only (wrong results): split tiles read B fragments for the first tiles only
#endif
#ifndef RMX_DIAG_NODMA
#define RMX_DIAG_NODMA 0  // timing probe only (wrong results): the plain split loop issues no DMAs after its prologue
#endif
#ifndef RMX_BF_PF
#define RMX_BF_PF 3  // bf16 fast tiles: B fragments read this many column tiles ahead
#endif

enum AMode : int { kDenseA = 0, kGatherK16 = 1, kGatherAny = 2, kCinOuter = 3 };
enum EpiMode : int { kEpiRelu = 0, kEpiOutput = 1, kEpiCin = 2 };

struct GemmArgs {
  int M, K, Kpad, Npad;
  const float* A;  // kDenseA: [M][lda]
  int lda;
  AGatherArgs ga;  // gather modes (ids, table, F, k); kCinOuter: ids, table, F, k of x0
  // kCinOuter
  const float* u_prev;  // [M][ldu] previous CIN maps, nullptr for the first layer (u = x0)
  int ldu, XS, cin_first;
  const int* cmap;  // kPrecS3 chunk map (CinLayer::cmap, staged in LDS), nullptr: chunk c16 = hc * F + f
  int ncmap;
  int cin_pair_hc;  // kPrecS3 without cmap: the h-chunk whose chunks carry two fields (-1: none)
  const float* Wp;     // [Kpad/16][Npad][16]
  const float* bias;   // [Npad]
  float* C;            // kEpiRelu / kEpiCin (u_out, may be null): [M][ldc]
  int ldc;
  OutArgs oa;          // kEpiOutput
  const float* wo;     // kEpiCin: [Npad] slice of the output Linear
  float* rowdot;       // kEpiCin: [M]
  float* xcol;         // kEpiRelu: raw extra columns n >= xn_main -> xcol[m * xld + n - xn_main] (DCN cross)
  int xn_main, xld;
  int prio;            // 1: the first half of the block's waves issue at raised priority (s_setprio)
  int cols32;          // kPrecS3 dense A: 32-column blocks (small launch batches, k_gemm_s3.hip s3_cols)
  int nt_store;        // 1: stored activations use non-temporal stores (knob "gemm_nt_store")
  // DeepFM first order + FM fused into tower layer 1 (kGatherK16 + kPrecS3, column slice 0): the A
  // tiles that stream through LDS are the gathered field rows, so the FM sums ride along and
  // fm_y[m] = y1 + y2 (bit-identical to encoder_k16_kernel<1>: same fp32 order, no contraction).
  // Without the FM sums (fm_sums = 0) the same epilogue gives the first order alone (y1, the other
  // models' Scatter term, bit-identical to encoder_k16_kernel<0>) for any k = 16 gather layer 1.
  const void* fm_w;    // first-order weights [V] (bf16 when fm_w_bf16), weight of id at fm_w[id << fm_wsh]
  int fm_w_bf16, fm_sums, fm_wsh;
  int gsh;             // kGatherK16: log2 of the table's row stride ga.ld (row of id at table + (id << gsh))
  int fm_add;          // 1: fm_y already holds y1 (a first-order kernel ran): fm_y = fm_y + y2
  float* fm_y;         // [M], nullptr = off
  // kEpiRelu variants for the backward's dX = dPre W (train.hip): raw = store acc (+ bias when
  // bias != nullptr) without the ReLU; mask [M][ldmask]: zero the entries whose mask is <= 0 (the
  // ReLU backward of the layer below, fused)
  int raw;
  const float* mask;
  int ldmask;
  // DeepFM training, dX of tower layer 1 written straight as the embedding gradient (train.hip): the
  // stored value becomes dx + dz[m] * (s[m][j] - x[m][n]) / 16 (emb_grad_kernel's FM term, same
  // arithmetic; j = n mod 16), with x [M][eg_ldx] the gathered rows and s [M][16] the FM sums
  const float* eg_x;
  const float* eg_s;
  const float* eg_dz;
  int eg_ldx;
};

template <int V>
using IC = std::integral_constant<int, V>;

constexpr int kFmMaxF = 40;  // fused FM: fields per sample it handles (F = 39 at the headline config)

// FM sums of one A fragment pair (fields 2c, 2c + 1; j = 4g .. 4g + 3): s += e, q += e * e in field
// order, without FMA contraction (SecondOrderEncoder.scala:19-34, the oracle's order)
__device__ __forceinline__ void fm_accum(const f32x4& a0, const f32x4& a1, f32x4& fs, f32x4& fq) {
#pragma clang fp contract(off)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    fs[t] = fs[t] + a0[t];
    fq[t] = fq[t] + a0[t] * a0[t];
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    fs[t] = fs[t] + a1[t];
    fq[t] = fq[t] + a1[t] * a1[t];
  }
}

// Block tiling: WM x WN waves; a wave owns MT*16 rows x NTW*16 columns (MT*NTW accumulator
// tiles); the block spans BM = WM*MT*16 rows and BN = WN*NTW*16 columns.  BKC 16-wide K chunks per
// LDS stage.  OCC = minimum waves per SIMD the register allocation must allow (launch bounds).
template <int MT_, int NTW_, int WM_, int WN_, int BKC_, int OCC_, int RING_ = 0, int STAG_ = 0, int FAST_ = 0>
struct Tile {
  // RING > 0: LDS-DMA (global_load_lds_dwordx4) ring of RING one-chunk stages, RING - 1 chunks in
  // flight, counted vmcnt + one raw barrier per chunk (needs BKC == 1); 0: register-staged double buffer
  // STAG (kPrecS3, RING == 2): the two waves of each SIMD run half a K step apart (staggered loop below)
  static constexpr int MT = MT_, NTW = NTW_, WM = WM_, WN = WN_, BKC = BKC_, OCC = OCC_, RING = RING_;
  static constexpr int STAG = STAG_;
  // FAST (kPrecBF16 ring tiles): the branch-free DMA issue and MFMA step of the split GEMM, applied
  // to bf16 operands (kPrecS3 tiles always run it)
  static constexpr int FAST = FAST_;
  static constexpr int NBUF = RING > 0 ? RING : 2;  // stage buffers in LDS
  static constexpr int NW = WM * WN, NTHR = NW * 64, NT = NTW * WN;
  static constexpr int BM = WM * MT * 16, BN = NT * 16;
};

// Operand precision of a GEMM instantiation:
//   kPrecF32   fp32 operands on v_mfma_f32_16x16x4_f32 (exact fp32 FMA chain);
//   kPrecBF16  bf16 operands on v_mfma_f32_16x16x32_bf16 (the bf16 configuration, configs[4]);
//   kPrecS3    fp32 operands computed on v_mfma_f32_16x16x32_bf16 through an exact 3-way bf16 split:
//              x = hi + mid + lo (each bf16, exact for every normal fp32), x*y summed over the six
//              products hi*hi, hi*mid, mid*hi, hi*lo, lo*hi, mid*mid.  |mid| <= 2^-8 |x| and
//              |lo| <= 2^-17 |x|, so the dropped terms are <= (2^-24 + 2^-34) |x y| (the size of
//              one fp32 rounding) and every kept product is exact in the fp32 accumulator: the
//              result is fp32-accurate at 6 x 16 / (8 x 32) = 3/8 of the fp32 MFMA cycles.  The weights are pre-split into three bf16 planes (W3); the A operand
//              is split in registers.
enum Prec : int { kPrecF32 = 0, kPrecBF16 = 1, kPrecS3 = 2 };

// kPrecS3 layer-1 gathers with an explicit id array: the ids of the next stages stream into a small
// LDS ring by DMA (2 slots x 2 fields x BM) instead of a [BM][F] id tile, so a BM = 256 ring fits
template <class T, int AMODE, int PREC>
constexpr bool kIdRing = AMODE == kGatherK16 && PREC == kPrecS3 && T::RING == 2 && T::MT >= 2;
// 2-deep ring kernels of k = 16 gathers in 32-wide K steps (two fields per step): the first-order
// weights of each step's (row, field) pairs can ride the ring ([2 slots][2 fields][BM] elements)
template <class T, int AMODE, int PREC>
constexpr bool kWRing = AMODE == kGatherK16 && (PREC == kPrecS3 || (PREC == kPrecBF16 && !T::FAST)) && T::RING == 2;
// the branch-free ring path (padded stages, every wave the same DMA instructions every step)
template <class T, int PREC>
constexpr bool kFastRing = T::RING > 0 && (PREC == kPrecS3 || (PREC == kPrecBF16 && T::FAST));

template <class T, int AMODE, int PREC = kPrecF32>
struct StageGeom {
  // kPrecS3: one stage = one 32-wide K step: A as two fp32 16-wide chunks [2][BM], B as the three
  // bf16 planes [3][BN] (each a 64-B row of 32 values)
  static constexpr int AROWS = AMODE != kCinOuter ? T::BM * (PREC == kPrecS3 ? 2 : T::BKC) : 0;
  static constexpr int ROWS = AROWS + T::BN * (PREC == kPrecS3 ? 3 : T::BKC);  // 64-B rows per stage
  // kPrecS3 ring stages are padded to whole DMA instructions per wave (16 rows each), so every wave
  // issues the same instructions every step with no per-wave branch (the padding rows take zeros)
  static constexpr int NINS = ROWS / 16;
  static constexpr int PADROWS = kFastRing<T, PREC> ? 16 * (((NINS + T::NW - 1) / T::NW) * T::NW - NINS) : 0;
  static constexpr int FLOATS = (ROWS + PADROWS) * 16;
};

// Epilogue slab geometry: each wave transposes NTH of its column tiles at a time through a
// private [RW][LD] fp32 slab carved from the (then idle) stage buffers, or more LDS if needed.
template <class T, int STAGE_FLOATS>
struct EpiGeom {
  static constexpr int RW = T::MT * 16;
  static constexpr int WF = (T::NBUF * STAGE_FLOATS) / T::NW;
  static constexpr int NTH0 = (WF / RW - 4) / 16;
  static constexpr int NTH = NTH0 < T::NTW ? (NTH0 < 1 ? 1 : NTH0) : T::NTW;
  static constexpr int LD = NTH * 16 + 4;  // == 4 mod 8: the two 16-lane halves of a write hit disjoint banks
  static constexpr int FLOATS = RW * LD * T::NW;
};

// LDS DMA (global_load_lds, `BYTES` per lane; lane L lands at dst + BYTES * L) issued through inline asm.
// With the builtin the compiler counts the DMA as an LGKM event of unknown order, so every later wait for
// an LDS read becomes lgkmcnt(0) and drains the prefetched fragments (checked on gfx950 ISA); hidden in
// asm, the reads keep their counted waits.  The kernels that use it order the DMAs themselves (explicit
// vmcnt waits + barriers) and issue no compiler-visible vector-memory loads in their loops.  M0 is an asm
// operand ("{m0}"): the compiler writes it before the asm and knows it holds the LDS address after it
// (a hand-written s_mov_b32 m0 inside the asm was invisible to the register allocator).
#ifndef RMX_LDS_DMA_BUILTIN
#define RMX_LDS_DMA_BUILTIN 0  // (1: the builtin, timing A/B builds only)
#endif
template <int BYTES>
__device__ __forceinline__ void lds_dma(const void* src, const void* dst) {
#if RMX_LDS_DMA_BUILTIN
  __attribute__((address_space(3))) void* d = (__attribute__((address_space(3))) void*)(uintptr_t)(unsigned)(uintptr_t)dst;
  if constexpr (BYTES == 16)
    __builtin_amdgcn_global_load_lds(src, d, 16, 0, 0);
  else if constexpr (BYTES == 4)
    __builtin_amdgcn_global_load_lds(src, d, 4, 0, 0);
  else
    __builtin_amdgcn_global_load_lds(src, d, 2, 0, 0);
  return;
#endif
  // (the low 32 bits of a generic pointer into LDS are the LDS address; the address-space cast's null
  // check tripped an instruction-selection bug, "V_CMP_NE_U32 ... src_shared_base")
  const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(dst));
  if constexpr (BYTES == 16)
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(a) : "memory");
  else if constexpr (BYTES == 4)
    asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "{m0}"(a) : "memory");
  else
    asm volatile("s_nop 0\n\tglobal_load_lds_ushort %0, off" ::"v"(src), "{m0}"(a) : "memory");
}

// x (8 fp32 as two float4) = hi + mid + lo exactly, each a bf16x8 (kPrecS3)
__device__ __forceinline__ void split3(const f32x4& x0, const f32x4& x1, bf16x8& hi, bf16x8& mi, bf16x8& lo) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float v = q < 4 ? x0[q & 3] : x1[q & 3];
    const __bf16 h = (__bf16)v;
    const float r = v - (float)h;
    const __bf16 m = (__bf16)r;
    hi[q] = h;
    mi[q] = m;
    lo[q] = (__bf16)(r - (float)m);
  }
}

template <class T, int AMODE, int EPI, int PREC>
__global__ __launch_bounds__(T::NTHR, T::OCC) void gemm_kernel(GemmArgs p) {
  // kPrecBF16: bf16 operands (v_mfma_f32_16x16x32_bf16, K chunk of 32 per 64-B row), fp32
  // accumulate, bf16 stored activations; kPrecF32: fp32 throughout (v_mfma_f32_16x16x4_f32, K
  // chunk 16); kPrecS3: fp32 A chunks of 16 (two per stage), three bf16 B planes of 32, fp32
  // stored activations.  A "chunk" c below is a K step of KC elements (32 for kPrecS3).
  constexpr bool BF = PREC == kPrecBF16, S3 = PREC == kPrecS3;
  constexpr int KC = (BF || S3) ? 32 : 16;       // K elements per step
  constexpr int KCA = BF ? 32 : 16, KSA = KCA / 4;  // A elements per 64-B row / per 16-B slot
  static_assert(!BF || AMODE != kCinOuter, "CIN has no bf16 configuration");
  static_assert(!S3 || T::BKC == 1, "kPrecS3 stages one K step at a time");
  constexpr int MT = T::MT, NTW = T::NTW, WN = T::WN, BKC = T::BKC;
  constexpr int BM = T::BM, BN = T::BN, NTHR = T::NTHR;
  constexpr bool A_LDS = AMODE != kCinOuter;
  using SG = StageGeom<T, AMODE, PREC>;
  constexpr int AROWS = SG::AROWS, ROWS = SG::ROWS, STAGE = SG::FLOATS;
  constexpr int ITEMS = ROWS * 4;  // float4 items per stage
  constexpr int PER = (ITEMS + NTHR - 1) / NTHR;

  // The DMA fill sources for out-of-range entries.  Under -fPIC a global's address comes from the GOT;
  // left alone, the compiler rematerialises it inside the MFMA stream as s_getpc + s_load +
  // s_waitcnt lgkmcnt(0) per DMA, which also drains the prefetched LDS fragment reads.  The empty
  // asm makes each address an opaque value computed once (kept in SGPRs).
  const float* zero16 = g_rmx_zero16;
  const int* neg1 = g_rmx_neg1;
  asm volatile("" : "+s"(zero16));
  asm volatile("" : "+s"(neg1));
#if RMX_GEMM_DIAG & 256
  const unsigned long long blk_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  constexpr int RING = T::RING;
  static_assert(RING == 0 || BKC == 1, "the LDS-DMA ring stages one K chunk at a time");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lds0 = smem;
  float* lds1 = smem + STAGE;
  float* extra = smem + T::NBUF * STAGE;  // gather: int ids [BM][F]; CIN: x0 [BM][XS]
  int* sids = reinterpret_cast<int*>(extra);

  // wid through readfirstlane: the compiler then treats everything derived from it as scalar
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int M = p.M;
  // XCD-aware block order for a layer in two column slices (kPrecS3, N = 400): blocks are dealt to
  // the 8 XCDs round-robin in linear order, so linear ids L and L + 8 land on the same XCD back to
  // back; map them to the two slices of one M block so the second slice's A rows (gathered table
  // rows or the previous activations) come from that XCD's L2 instead of HBM.
  int bx = blockIdx.x, by = blockIdx.y;
  if (gridDim.y == 2 && (gridDim.x & 7) == 0) {
    const int L = blockIdx.x + blockIdx.y * gridDim.x;
    const int j = L >> 3;
    by = j & 1;
    bx = (j >> 1) * 8 + (L & 7);
  }
  const int m0 = bx * BM;
  const int n0 = by * BN;
  const int nchunks = p.Kpad / KC;
  const int nstages = (nchunks + BKC - 1) / BKC;
  const int F = p.ga.F;

  constexpr bool IDRING = kIdRing<T, AMODE, PREC>;
  constexpr bool FAST = kFastRing<T, PREC>;
  int* idring = reinterpret_cast<int*>(extra);  // IDRING: [2 slots][2 fields][BM] ids
  // WRING + fused first order: the first-order weights of each step's (row, field) pairs ride the
  // DMA ring ([2 slots][2 fields][BM] table elements after the ids), summed per step in field order
  constexpr bool WRING = kWRing<T, AMODE, PREC> && EPI == kEpiRelu;
  float* wring = IDRING ? reinterpret_cast<float*>(extra) + 4 * BM : reinterpret_cast<float*>(sids + BM * F);
  if constexpr ((AMODE == kGatherK16 || AMODE == kGatherAny) && !IDRING) {
    for (int i = tid; i < BM * F; i += NTHR) {
      const int r = i / F, f = i - r * F;
      const int m = m0 + r;
      int id = 0;
      if (m < M) id = p.ga.ids ? p.ga.ids[(int64_t)m * F + f] : m * F + f;
      sids[i] = id;
    }
    __syncthreads();
  }
  if constexpr (AMODE == kCinOuter) {
    // x0 tile: x0s[r][f] = e[b, f, j] for row m0 + r = b*k + j, zero padded to XS columns
    const int k = p.ga.k, XS = p.XS;
    for (int i = tid; i < BM * XS; i += NTHR) {
      const int j = i % k;
      const int rest = i / k;
      const int f = rest % XS;
      const int rb = rest / XS;
      const int r = rb * k + j;
      if (r >= BM) continue;
      const int m = m0 + r;
      float v = 0.f;
      if (f < F && m < M) {
        const int b = m / k;
        const int id = p.ga.ids ? p.ga.ids[(int64_t)b * F + f] : b * F + f;
        v = p.ga.table[(int64_t)id * p.ga.ld + j];
      }
      extra[r * XS + f] = v;
    }
    // the chunk map after the x0 tile (read wave-uniformly in the MFMA loop: an LDS broadcast, no
    // vector-memory op among the counted DMAs)
    if (S3 && p.cmap)
      for (int i = tid; i < p.ncmap; i += NTHR) reinterpret_cast<int*>(extra + BM * XS)[i] = p.cmap[i];
    __syncthreads();
  }

  // Staggered issue (knob "gemm_prio"): waves w and w + NW/2 share a SIMD; giving the first half
  // priority lets it finish its post-barrier VALU work (A split, addressing) and start its MFMAs
  // while the partner's VALU runs in the MFMA shadow.
  // prio 1: the first half at raised priority; prio 2: the second-dispatched half (waves NW/2..NW-1,
  // the arbitration losers: MI355X_MICROARCH.md "two waves per SIMD" item 4) at priority 1
  if (p.prio == 1 && wid < T::NW / 2) __builtin_amdgcn_s_setprio(2);
  if (p.prio == 2 && wid >= T::NW / 2) __builtin_amdgcn_s_setprio(1);
  constexpr bool FM = AMODE == kGatherK16 && EPI == kEpiRelu;  // first order (+ FM sums on kPrecS3)
  constexpr bool FMS = FM && S3;
  const bool fm_on = FM && p.fm_y != nullptr && by == 0;
  const bool fm_sums = FMS && fm_on && p.fm_sums;
  const bool wfuse = WRING && fm_on && !p.fm_add;
  float y1acc[WRING ? MT : 1];
#pragma unroll
  for (int i = 0; i < (WRING ? MT : 1); ++i) y1acc[i] = 0.f;
  f32x4 fm_s[FMS ? MT : 1], fm_q[FMS ? MT : 1];
#pragma unroll
  for (int i = 0; i < (FMS ? MT : 1); ++i) fm_s[i] = fm_q[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc[MT][NTW];
#if RMX_GEMM_DIAG & 8
  // DIAG & 16: only CIN launches record (xDeepFM's last split-GEMM launch is a tower layer)
  // DIAG & 64: dense-A tower launches record (the last one is the output layer); & 128: gathered
  // layer 1; else the CIN layers (K > 100 steps)
  constexpr bool kDiagSel = (RMX_GEMM_DIAG & 64)    ? AMODE == kDenseA
                            : (RMX_GEMM_DIAG & 128) ? AMODE == kGatherK16
                                                    : (!(RMX_GEMM_DIAG & 16) || AMODE == kCinOuter);
  const bool dmark = blockIdx.x == 0 && blockIdx.y == 0 && (wid == 0 || wid == T::NW / 2) && kDiagSel;
  unsigned long long dsum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dlast = __builtin_amdgcn_s_memtime();
  const unsigned long long dt0 = dlast, drt0 = __builtin_amdgcn_s_memrealtime();
#endif
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Global source of logical 16-B slot g of stage row `row` (A rows first: [BKC or 2][BM], then
  // B rows [BKC or 3][BN]) for stage st; nullptr = zeros (out-of-range rows, K padding).
  auto src_of = [&](int row, int g, int st) -> const void* {
    if (row < AROWS) {
      const int cc = row / BM, r = row - cc * BM;
      const int c = S3 ? 2 * st + cc : st * BKC + cc;  // A chunk of KCA elements
      const int m = m0 + r;
      const int kk = c * KCA + g * KSA;
      if (m >= M || kk >= p.K) return nullptr;
      if constexpr (AMODE == kGatherK16) {
        // fp32: chunk c = field c; bf16: chunk c = fields 2c, 2c+1 (two 32-B rows)
        const int f = BF ? 2 * c + (g >> 1) : c;
        const int id = sids[r * F + f];
        return BF ? (const void*)(reinterpret_cast<const bf16_t*>(p.ga.table) + ((int64_t)id << p.gsh) + (g & 1) * 8)
                  : (const void*)(p.ga.table + ((int64_t)id << p.gsh) + g * 4);
      } else if constexpr (AMODE == kGatherAny) {
        const int f = kk / p.ga.k, j = kk - f * p.ga.k;
        const int id = sids[r * F + f];
        return BF ? (const void*)(reinterpret_cast<const bf16_t*>(p.ga.table) + (int64_t)id * p.ga.ld + j)
                  : (const void*)(p.ga.table + (int64_t)id * p.ga.ld + j);
      } else {
        return BF ? (const void*)(reinterpret_cast<const bf16_t*>(p.A) + (int64_t)m * p.lda + kk)
                  : (const void*)(p.A + (int64_t)m * p.lda + kk);
      }
    }
    const int rb = row - AROWS;
    const int cc = rb / BN, n = rb - cc * BN;
    if constexpr (S3)  // plane cc of step st: W3 [steps][3][Npad][32] bf16
      return reinterpret_cast<const bf16_t*>(p.Wp) + ((int64_t)(st * 3 + cc) * p.Npad + n0 + n) * 32 + g * 8;
    const int c = st * BKC + cc;
    if (c >= nchunks) return nullptr;
    return BF ? (const void*)(reinterpret_cast<const bf16_t*>(p.Wp) + ((int64_t)c * p.Npad + n0 + n) * 32 + g * 8)
              : (const void*)(p.Wp + ((int64_t)c * p.Npad + n0 + n) * 16 + g * 4);
  };

  float4 stage[PER];
  // item i of a stage: row = i >> 2, slot g = i & 3
  auto gload = [&](int st) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = tid + q * NTHR;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int row = i >> 2, g = i & 3;
      if (row < ROWS) {
        const void* src = src_of(row, g, st);
        if (src) v = *reinterpret_cast<const float4*>(src);
      }
      stage[q] = v;
    }
  };
  auto sstore = [&](float* buf) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = tid + q * NTHR;
      const int row = i >> 2, g = i & 3;
      if (row < ROWS) {
        const int lrow = row < AROWS ? (row % BM) : ((row - AROWS) % BN);
        *reinterpret_cast<float4*>(buf + row * 16 + swz_slot(lrow, g) * 4) = stage[q];
      }
    }
  };

  const int g = lane >> 4, r16 = lane & 15;
  int arow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) arow[i] = wm * MT * 16 + i * 16 + r16;
  const int bt0 = wn * NTW;  // first column tile of this wave
  // w-ring element e of slot (c & 1): an fp32 weight, or a bf16 one zero-extended to a dword (a
  // 2-byte LDS DMA writes lane L at base + 4 L, tools/probe/glds_sizes.hip), widened exactly
  auto wget = [&](int c, int part, int r) -> float {
    const int e = ((c & 1) * 2 + part) * BM + r;
    return (!S3 && p.fm_w_bf16) ? __uint_as_float(__float_as_uint(wring[e]) << 16) : wring[e];
  };
  // the weights of fields 2c, 2c + 1 of this lane's rows, in field order
  auto wsum = [&](int c) {
#pragma unroll
    for (int i = 0; i < (WRING ? MT : 1); ++i) {
      y1acc[i] += wget(c, 0, arow[i]);
      y1acc[i] += wget(c, 1, arow[i]);
    }
  };

  // kCinOuter: the row's u[h-chunk] for the current hc, reloaded when hc changes (kPrecS3: one
  // cache per half of the 32-wide step, whose two 16-wide chunks may sit in different h-chunks)
  constexpr int NU = S3 ? 2 : 1;
  float4 uf[NU][MT];
  int cur_hc[NU];
#pragma unroll
  for (int h = 0; h < NU; ++h) cur_hc[h] = -1;
  // key = hc * 2 + pair (cin_chunk): lane group g's maps 16 hc + 4 g .. (pair: 16 hc + 4 (g & 1) ..)
  auto load_u = [&](int h, int key) {
    const int col = (key >> 1) * 16 + ((key & 1) ? (g & 1) * 4 : g * 4);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (p.cin_first) {
        uf[h][i] = *reinterpret_cast<const float4*>(extra + arow[i] * p.XS + col);
      } else {
        const int m = m0 + arow[i];
        uf[h][i] = m < M ? *reinterpret_cast<const float4*>(p.u_prev + (int64_t)m * p.ldu + col)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    cur_hc[h] = key;
  };
  // CIN A fragment of 16-wide chunk c16 (= hc * F + f): a = x0[row][f] * u[row][16 hc + 4 g ..]
  // c16 / F for the (wave-uniform) chunk index: q = floor(c16 * ceil(2^32 / F) / 2^32) is exact for
  // c16, F < 2^16 -- two scalar multiplies instead of the generic division's VALU sequence
  const uint64_t fmagic = ((1ull << 32) + (uint64_t)F - 1) / (uint64_t)(F > 0 ? F : 1);
#ifndef RMX_CIN_DIVF
#define RMX_CIN_DIVF 1  // (0: the generic division, timing A/B only)
#endif
  auto div_f = [&](int c16) -> int {
    return RMX_CIN_DIVF ? (int)(((uint64_t)(uint32_t)c16 * fmagic) >> 32) : c16 / F;
  };
  // chunk c16 -> this lane's field f and the u-slice key hc * 2 + pair.  With a chunk map (kPrecS3)
  // the wave-uniform entry comes from LDS; a pair entry gives lane groups 2-3 the next field
  const int* lmap = reinterpret_cast<const int*>(extra + BM * p.XS);
  auto cin_chunk = [&](int c16, int& f, int& key) {
    if (S3 && p.cmap) {
      const int e = __builtin_amdgcn_readfirstlane(c16 * 16 < p.K ? lmap[c16] : 0);
      const int pr = (e >> 30) & 1;
      f = (e & 0xffff) + (pr ? (g >> 1) : 0);
      key = ((e >> 16) & 0x3fff) * 2 + pr;
    } else {
      // the same order in closed form for a map without the triangle: h-chunk hc = c16 / F plain,
      // except a paired last h-chunk p.cin_pair_hc (its chunk j carries fields 2j, 2j + 1)
      const int hc = div_f(c16);
      const int j = c16 - hc * F;
      const int pr = S3 && hc == p.cin_pair_hc ? 1 : 0;
      f = pr ? 2 * j + (g >> 1) : j;
      key = hc * 2 + pr;
    }
  };
  // the x0 scalars of chunk c16 (LDS) and its u-slice key, decoded once: the step that uses them reads the
  // key from here instead of decoding the chunk again at its head (a chunk-map LDS read, or div_f, ahead of
  // the A generation)
  auto cin_x0 = [&](int c16, float* xv, int& key) {
    int f;
    cin_chunk(c16, f, key);
#pragma unroll
    for (int i = 0; i < MT; ++i) xv[i] = c16 * 16 < p.K ? extra[arow[i] * p.XS + f] : 0.f;
  };
  auto cin_a_x = [&](int h, int c16, const float* xv, int key, f32x4* a) {
    if (c16 * 16 >= p.K) {
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    if (key != cur_hc[h]) load_u(h, key);
#pragma unroll
    for (int i = 0; i < MT; ++i)
      a[i] = f32x4{xv[i] * uf[h][i].x, xv[i] * uf[h][i].y, xv[i] * uf[h][i].z, xv[i] * uf[h][i].w};
  };
  auto cin_a = [&](int h, int c16, f32x4* a) {
    float xv[MT];
    int key;
    cin_x0(c16, xv, key);
    cin_a_x(h, c16, xv, key, a);
  };
  // kPrecS3: the x0 scalars (and u-slice keys) of the next K step, read during this step's MFMAs (x0 is
  // static in LDS)
  float x0q[2][MT];
  int kq[2] = {0, 0};

  // kPrecS3: one 32-wide K step c.  Lane group g holds, at bf16 position 4h + q of its fragment,
  // K index 16h + 4g + q of the step (fp32 chunk 2c + h, slot g) -- the order W3 is packed in.
  // DMA instructions per wave per stage (ring kernels); kPrecS3 spreads them over the MFMA tiles
  constexpr int kQID = IDRING ? (2 * BM / 64 + T::NW - 1) / T::NW : 0;  // id-ring DMAs per wave
  constexpr int kQW = WRING ? (2 * BM / 64 + T::NW - 1) / T::NW : 0;    // w-ring DMAs per wave
  constexpr int kIPW = kQID + kQW + (ROWS / 16 + T::NW - 1) / T::NW;
  auto compute_step_s3 = [&](const float* cur, int c, auto&& dma, auto&& dpre) {
    f32x4 a0[MT], a1[MT];
    if constexpr (A_LDS) {
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int o = arow[i] * 16 + swz_slot(arow[i], g) * 4;
        a0[i] = *reinterpret_cast<const f32x4*>(cur + o);
        a1[i] = *reinterpret_cast<const f32x4*>(cur + BM * 16 + o);
      }
      // unconditional (no branch inside the MFMA loop); read only when the launch asked for them
      if constexpr (FMS)
#pragma unroll
        for (int i = 0; i < MT; ++i) fm_accum(a0[i], a1[i], fm_s[i], fm_q[i]);
      if constexpr (WRING) wsum(c);
    } else {
      if (c == 0) {
        cin_x0(0, x0q[0], kq[0]);
        cin_x0(1, x0q[1], kq[1]);
      }
      cin_a_x(0, 2 * c, x0q[0], kq[0], a0);
      cin_a_x(1, 2 * c + 1, x0q[1], kq[1], a1);
    }
    RMX_TMARK(3);  // 3: A fragments (LDS reads / CIN generation)
    bf16x8 ah[MT], am[MT], al[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if constexpr (RMX_GEMM_DIAG & 1) {
        ah[i] = __builtin_bit_cast(bf16x8, a0[i]);
        am[i] = __builtin_bit_cast(bf16x8, a1[i]);
        al[i] = ah[i];
      } else {
        split3(a0[i], a1[i], ah[i], am[i], al[i]);
      }
    }
    RMX_TMARK(4);  // 4: split
    const float* Bt = cur + AROWS * 16;  // planes [3][BN] of 64-B rows
    // the three plane fragments of column tile t
    auto ldb = [&](int t, f32x4* b) {
      const int row = (bt0 + t) * 16 + r16;
      const int o = row * 16 + swz_slot(row, g) * 4;
      b[0] = *reinterpret_cast<const f32x4*>(Bt + o);
      b[1] = *reinterpret_cast<const f32x4*>(Bt + BN * 16 + o);
      b[2] = *reinterpret_cast<const f32x4*>(Bt + 2 * BN * 16 + o);
    };
    // software pipeline: the fragments of tile t + PF are read while tile t's MFMAs run, so each
    // MFMA group waits only for its own reads (counted lgkmcnt), not for a drained LDS queue
    constexpr int PF = 2;
    f32x4 bq[PF + 1][3];
    if (0 < kIPW) dpre(0);
#pragma unroll
    for (int t = 0; t < PF && t < NTW; ++t) ldb(t, bq[t]);
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      if (t + PF < NTW && !RMX_DIAG_NOB) ldb(t + PF, bq[(t + PF) % (PF + 1)]);
      // one of the next stage's DMA instructions per tile: a DMA issue can stall the wave for ~200
      // cycles (vector-memory queue), which here overlaps the partner wave's MFMAs instead of
      // idling the SIMD in a separate post-barrier phase
      if (t < kIPW && !RMX_DIAG_NODMA) dma(t);
      // the LDS-held operand (a ring id) of the next DMA is read one MFMA group ahead of its use
      if (t + 1 < kIPW) dpre(t + 1);
      if constexpr (!A_LDS)
        if (t == 0) {
          cin_x0(2 * c + 2, x0q[0], kq[0]);
          cin_x0(2 * c + 3, x0q[1], kq[1]);
        }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this tile's MFMAs
      const f32x4* b = bq[t % (PF + 1)];
      const bf16x8 bh = __builtin_bit_cast(bf16x8, b[0]);
      const bf16x8 bm = __builtin_bit_cast(bf16x8, b[1]);
      const bf16x8 bl = __builtin_bit_cast(bf16x8, b[2]);
      if constexpr (RMX_GEMM_DIAG & 4) {
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i][t] += b[0] + b[1] + b[2] + __builtin_bit_cast(f32x4, ah[i]);
        continue;
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        f32x4 d = acc[i][t];
        // smallest terms first
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bm, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bh, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bm, d, 0, 0, 0);
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, d, 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = NTW; q < kIPW; ++q)
      if (!RMX_DIAG_NODMA) dma(q);
    RMX_TMARK(5);  // 5: MFMA section (issue)
  };

  // kPrecBF16 fast tiles: one 32-wide K step c -- one bf16 A fragment per row tile (LDS), the B
  // fragment of each column tile read PF tiles ahead, one MFMA per (row tile, column tile); the
  // next stages' DMAs ride one per MFMA group (same structure as compute_step_s3, 1/6 the MFMAs)
  auto compute_step_bf16 = [&](const float* cur, int c, auto&& dma) {
    bf16x8 a[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
      a[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const f32x4*>(cur + arow[i] * 16 + swz_slot(arow[i], g) * 4));
    const float* Bt = cur + AROWS * 16;
    auto ldb = [&](int t) -> f32x4 {
      const int row = (bt0 + t) * 16 + r16;
      return *reinterpret_cast<const f32x4*>(Bt + row * 16 + swz_slot(row, g) * 4);
    };
    constexpr int PF = RMX_BF_PF < NTW ? RMX_BF_PF : NTW;
    f32x4 bq[PF + 1];
#pragma unroll
    for (int t = 0; t < PF && t < NTW; ++t) bq[t] = ldb(t);
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      if (t + PF < NTW) bq[(t + PF) % (PF + 1)] = ldb(t + PF);
      if (t < kIPW) dma(t);
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 b = __builtin_bit_cast(bf16x8, bq[t % (PF + 1)]);
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][t], 0, 0, 0);
    }
#pragma unroll
    for (int q = NTW; q < kIPW; ++q) dma(q);
  };

  // one K chunk c of the stage image at `cur` (chunk slot cc inside the stage)
  // dma(q): issue this wave's q-th DMA instruction of the next stage (ring kernels), spread over the
  // MFMA groups so its issue stall overlaps MFMAs (a no-op for the register-staged pipeline)
  auto compute_chunk = [&](const float* cur, int cc, int c, auto&& dma, auto&& dpre) {
    if constexpr (S3) {
      compute_step_s3(cur, c, dma, dpre);
    } else if constexpr (FAST) {
      compute_step_bf16(cur, c, dma);
    } else {
      const float* Bt = cur + AROWS * 16 + cc * BN * 16;
      f32x4 a[MT];
      if constexpr (A_LDS) {
        const float* At = cur + cc * BM * 16;
#pragma unroll
        for (int i = 0; i < MT; ++i)
          a[i] = *reinterpret_cast<const f32x4*>(At + arow[i] * 16 + swz_slot(arow[i], g) * 4);
        if constexpr (WRING)
          if (wfuse) wsum(c);
      } else {
        cin_a(0, c, a);
      }
      // groups of >= 4 independent accumulator tiles: consecutive MFMAs of one tile are a group
      // apart (>= 128 cycles), past the 40-cycle dependent latency of v_mfma_f32_16x16x4_f32
      constexpr int NG = NTW >= 4 ? NTW / 4 : 1;
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        const int j0 = gi * NTW / NG, j1 = (gi + 1) * NTW / NG;
#pragma unroll
        for (int q = gi * kIPW / NG; q < (gi + 1) * kIPW / NG; ++q) dma(q);
        f32x4 b[8];
#pragma unroll
        for (int t = 0; t < 8; ++t)
          if (j0 + t < j1) {
            const int row = (bt0 + j0 + t) * 16 + r16;
            b[t] = *reinterpret_cast<const f32x4*>(Bt + row * 16 + swz_slot(row, g) * 4);
          }
        if constexpr (BF) {
#pragma unroll
          for (int t = 0; t < 8; ++t)
            if (j0 + t < j1)
#pragma unroll
              for (int i = 0; i < MT; ++i)
                acc[i][j0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, a[i]), __builtin_bit_cast(bf16x8, b[t]), acc[i][j0 + t], 0, 0, 0);
        } else {
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
            for (int t = 0; t < 8; ++t)
              if (j0 + t < j1)
#pragma unroll
                for (int i = 0; i < MT; ++i)
                  acc[i][j0 + t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s4], b[t][s4], acc[i][j0 + t], 0, 0, 0);
        }
      }
    }
  };

  if constexpr (RING == 0) {
    gload(0);
    sstore(lds0);
    __syncthreads();
    for (int st = 0; st < nstages; ++st) {
      const float* cur = (st & 1) ? lds1 : lds0;
      float* nxt = (st & 1) ? lds0 : lds1;
      const bool more = st + 1 < nstages;
      if (more) gload(st + 1);
#pragma unroll
      for (int cc = 0; cc < BKC; ++cc) {
        const int c = st * BKC + cc;
        if (BKC > 1 && c >= nchunks) break;
        compute_chunk(cur, cc, c, [](int) {}, [](int) {});
      }
      if (more) sstore(nxt);
      __syncthreads();
    }
  } else {
    // LDS-DMA ring: wave-instruction ins of a chunk fills stage rows [16 ins, 16 ins + 16) (1 KiB);
    // lane L writes physical slot L&3 of row L>>2, so it loads logical slot (L&3) ^ key(row): the
    // swizzle goes on the source address, the LDS image stays lane-linear (guide rule 21).
    constexpr int NW = T::NW;
    constexpr int NINS = ROWS / 16;
    constexpr int IPW = (NINS + NW - 1) / NW;
    // DMAs this wave issues per chunk (kPrecS3: every wave IPW, padding included)
    const int my_n = FAST ? IPW : (wid < NINS ? (NINS - 1 - wid) / NW + 1 : 0);
    // A wave's instructions are the same every step (ins is wave-uniform), so the A / B region
    // and the chunk / plane of an instruction are scalar; dense A and B sources are a 32-bit
    // per-lane element offset plus a per-step stride (launch_cfg checks M * lda < 2^32).
    auto issue_one = [&](int c, int q) {
      float* buf = smem + (c % RING) * STAGE;
      {
        const int ins = wid + q * NW;
        if (q < IPW && ins < NINS) {
          const int row = ins * 16 + (lane >> 2), ps = lane & 3;
          const void* src;
          if (ins * 16 < AROWS) {
            const int cc = ins * 16 / BM;
            const int r = row - cc * BM, g = swz_slot(r, ps);
            if constexpr (AMODE == kDenseA) {
              const int m = m0 + r, kk = c * KC + cc * KCA + g * KSA;
              const uint32_t o = (uint32_t)m * (uint32_t)p.lda + (uint32_t)kk;
              src = (m < M && kk < p.K) ? (BF ? (const void*)(reinterpret_cast<const bf16_t*>(p.A) + o)
                                             : (const void*)(p.A + o))
                                        : (const void*)zero16;
            } else if constexpr (IDRING) {
              const int id = idring[((c & 1) * 2 + cc) * BM + r];
              src = id >= 0 ? (const void*)(p.ga.table + ((int64_t)id << p.gsh) + g * 4) : (const void*)zero16;
            } else {
              src = src_of(row, g, c);
              if (!src) src = zero16;
            }
          } else {
            const int cc = (ins * 16 - AROWS) / BN;
            const int n = row - AROWS - cc * BN, g = swz_slot(n, ps);
            if constexpr (S3) {
              src = reinterpret_cast<const bf16_t*>(p.Wp) +
                    ((uint32_t)((c * 3 + cc) * p.Npad + n0 + n) * 32u + (uint32_t)(g * 8));
            } else {
              src = BF ? (const void*)(reinterpret_cast<const bf16_t*>(p.Wp) +
                                       ((uint32_t)(c * p.Npad + n0 + n) * 32u + (uint32_t)(g * 8)))
                       : (const void*)(p.Wp + ((uint32_t)(c * p.Npad + n0 + n) * 16u + (uint32_t)(g * 4)));
            }
          }
          lds_dma<16>(src, buf + ins * 256);
        }
      }
    };
    // kPrecS3: the same DMA instruction q of source step cs into ring slot `slot`, with no branch:
    // whether q is an A or a B instruction is known at compile time (A rows are a whole number of
    // instructions per wave), the padding instruction of a ragged last q reads zeros into the
    // stage's padding rows, and the caller clamps cs to the last step instead of skipping it.
    // (Branches here split the MFMA stream into basic blocks and the compiler then drains every
    // prefetched LDS fragment read with lgkmcnt(0) at each join.)
    constexpr int AINS_ = AROWS / 16;
    // ring ids of DMA instruction q: A rows of source step cs (IDRING) / first-order weights of step c
    auto a_id = [&](int cs, int q) -> int {
      const int ins = wid + q * NW;
      const int row = ins * 16 + (lane >> 2), cc = ins * 16 / BM;
      return idring[((cs & 1) * 2 + cc) * BM + row - cc * BM];
    };
    auto w_id = [&](int c, int q) -> int {
      const int ins = wid + q * NW;
      const int v = ins * 64 + lane, part = v / BM, r = v - part * BM;
      if constexpr (IDRING) {
        return idring[((c & 1) * 2 + part) * BM + r];
      } else {
        const int f = 2 * c + part;
        return (f < F && m0 + r < M) ? sids[r * F + f] : -1;
      }
    };
    // get_id(): the ring id of an IDRING A instruction (read here, or one MFMA group earlier)
    auto issue_s3 = [&](int cs, int slot, int q, auto&& get_id) {
      if constexpr (FAST) {
        float* buf = smem + slot * STAGE;
        const int ins = wid + q * NW;
        const int row = ins * 16 + (lane >> 2), ps = lane & 3;
        const void* src;
        if ((q + 1) * NW <= AINS_ || (q * NW < AINS_ && ins < AINS_)) {
          const int cc = ins * 16 / BM;
          const int r = row - cc * BM, g = swz_slot(r, ps);
          if constexpr (AMODE == kDenseA) {
            const int m = m0 + r, kk = cs * KC + cc * KCA + g * KSA;
            const uint32_t o = (uint32_t)m * (uint32_t)p.lda + (uint32_t)kk;
            src = (m < M && kk < p.K) ? (BF ? (const void*)(reinterpret_cast<const bf16_t*>(p.A) + o) : (const void*)(p.A + o))
                                      : (const void*)zero16;
          } else if constexpr (IDRING) {
            const int id = get_id();
            src = id >= 0 ? (const void*)(p.ga.table + ((int64_t)id << p.gsh) + g * 4) : (const void*)zero16;
          } else {
            src = src_of(row, g, cs);
            if (!src) src = zero16;
          }
        } else {
          const int cc = (ins * 16 - AROWS) / BN;
          const int n = row - AROWS - cc * BN, g = swz_slot(n, ps);
          // kPrecS3: plane cc of step cs (W3 [steps][3][Npad][32]); bf16: W16 [chunks][Npad][32]
          src = reinterpret_cast<const bf16_t*>(p.Wp) +
                ((uint32_t)((cs * (S3 ? 3 : 1) + cc) * p.Npad + n0 + n) * 32u + (uint32_t)(g * 8));
          if ((q + 1) * NW > NINS) src = ins < NINS ? src : (const void*)zero16;  // padding instruction
        }
        lds_dma<16>(src, buf + ins * 256);
      }
    };
    auto issue = [&](int c) {
#pragma unroll
      for (int q = 0; q < IPW; ++q) {
        if constexpr (FAST)
          issue_s3(c, c % RING, q, [&] { return a_id(c, q); });
        else
          issue_one(c, q);
      }
    };
    // IDRING: the ids of fields 2c, 2c + 1 for the block's rows -> slot c & 1 (one dword per lane)
    auto issue_id = [&](int c, int q) {
      const int ins = wid + q * NW;
      if (kQID * NW == 2 * BM / 64 || ins < 2 * BM / 64) {
        const int v = ins * 64 + lane, part = v / BM, r = v - part * BM, m = m0 + r, f = 2 * c + part;
        const void* src = (m < M && f < F) ? (const void*)(p.ga.ids + (int64_t)m * F + f) : (const void*)neg1;
        lds_dma<4>(src, idring + (c & 1) * 2 * BM + ins * 64);
      }
    };
    // the first-order weights of stage c (ids of slot c & 1 landed, or the id tile) -> w slot c & 1,
    // one dword per lane (a 2-byte DMA of a bf16 weight fills the low half, zero-extended)
    auto issue_w = [&](int c, int q, auto&& get_id) {
      const int ins = wid + q * NW;
      if (kQW * NW == 2 * BM / 64 || ins < 2 * BM / 64) {
        const int id = get_id();
        const int e = (c & 1) * 2 * BM + ins * 64;
        if (!S3 && p.fm_w_bf16) {  // (kPrecS3 models have fp32 tables: launch_tower_s3 checks)
          const void* src = id >= 0 ? (const void*)(reinterpret_cast<const bf16_t*>(p.fm_w) + ((int64_t)id << p.fm_wsh))
                                    : (const void*)zero16;
          lds_dma<2>(src, wring + e);
        } else {
          // (kPrecS3 issues this unconditionally: zeros when the launch fuses no first order)
          const bool ok = id >= 0 && (!S3 || wfuse);
          const void* src = ok ? (const void*)(reinterpret_cast<const float*>(p.fm_w) + ((int64_t)id << p.fm_wsh))
                               : (const void*)zero16;
          lds_dma<4>(src, wring + e);
        }
      }
    };
    if constexpr (IDRING) {
#pragma unroll
      for (int q = 0; q < kQID; ++q) {
        issue_id(0, q);
        if (nchunks > 1) issue_id(1, q);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if constexpr (WRING)
      if (wfuse)
#pragma unroll
        for (int q = 0; q < kQW; ++q) issue_w(0, q, [&] { return w_id(0, q); });
    if constexpr (FAST) {
      // always RING - 1 stages (the loop's counted wait assumes RING - 2 younger ones in flight):
      // with fewer steps than that, the last step's sources fill the spare slots (never read)
      if (nchunks > 0)
        for (int c = 0; c < RING - 1; ++c) {
          const int cs = c < nchunks ? c : nchunks - 1;
#pragma unroll
          for (int q = 0; q < IPW; ++q) issue_s3(cs, c % RING, q, [&] { return a_id(cs, q); });
        }
    } else {
      for (int c = 0; c < RING - 1 && c < nchunks; ++c) issue(c);
    }
    int pend_id = -1;  // kPrecS3: the ring id of the next DMA, read one MFMA group ahead
    if constexpr (RING == 1) {
      // Single-buffered stage, two (or more) blocks per CU: each block loads a step, computes it,
      // and only then loads the next, so its own DMA latency and epilogue are exposed -- and covered
      // by the other resident block's MFMAs instead of by a second LDS stage (kPrecS3 only).
      static_assert(S3, "the single-stage loop is a split-GEMM tile");
      for (int c = 0; c < nchunks; ++c) {
        issue(c);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's DMAs of step c have landed
        compute_chunk(smem, 0, c, [](int) {}, [](int) {});
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave has read step c: the next issue may overwrite it
      }
    } else if constexpr (S3 && T::STAG) {
      // Staggered split-GEMM loop (two barriers per K step).  Waves w and w + NW/2 share a SIMD's
      // matrix pipe.  In the plain loop both reach the step barrier together and then both read
      // and split their A fragments (VALU + LDS latency) while the pipe idles.  Here the second
      // half (Y) runs its column tiles [NT1, NTW) one step late:
      //   phase 1 (bar0(c) .. bar1(c)):  X: prep(c), tiles [0, NT1) of step c
      //                                  Y: tiles [NT1, NTW) of step c - 1 (B of step c - 1)
      //   phase 2 (bar1(c) .. bar0(c+1)): X: tiles [NT1, NTW) of step c
      //                                  Y: prep(c), tiles [0, NT1) of step c
      // so each wave's prep overlaps its partner's MFMAs, and each phase carries one step's worth
      // of MFMAs per SIMD.  Y's split A of step c - 1 is still in its registers in phase 1 (no extra
      // registers: the accumulator of a tile is the same across steps).  The A rows, ids and
      // first-order weights of step c + 1 (their LDS slots were last read before bar0(c)) are
      // issued in phase 1; the B planes of step c + 1 go into the buffer Y reads in phase 1, so
      // they are issued after bar1(c) and have phase 2 to land (weights: L2 hits).
      static_assert(RING == 2 && BKC == 1, "the staggered loop runs on the 2-deep ring");
      constexpr int NT1 = (NTW + 1) / 2;
      constexpr int AINS = AROWS / 16;
      static_assert(AINS % NW == 0, "every wave issues the same number of A-region DMAs");
      constexpr int QA = AINS / NW;              // this wave's A-region DMAs: q in [0, QA)
      constexpr int NP1 = kQID + kQW + QA;       // phase-1 DMAs per wave
      constexpr int NP2 = IPW - QA;              // phase-2 (B-plane) DMAs per wave
      const bool late = wid >= NW / 2;
      bf16x8 ah[MT], am[MT], al[MT];
      auto dma1 = [&](int c, int q) {
        if (q < kQID) {
          if constexpr (IDRING) issue_id(c + 2, q);
        } else if (q < kQID + kQW) {
          if constexpr (WRING) issue_w(c + 1, q - kQID, [&] { return w_id(c + 1, q - kQID); });
        } else {
          const int cs = c + 1 < nchunks ? c + 1 : nchunks - 1;
          issue_s3(cs, (c + 1) & 1, q - kQID - kQW, [&] { return a_id(cs, q - kQID - kQW); });
        }
      };
      auto dma2 = [&](int c, int q) {
        const int cs = c + 1 < nchunks ? c + 1 : nchunks - 1;
        issue_s3(cs, (c + 1) & 1, QA + q, [&] { return a_id(cs, QA + q); });
      };
      // A fragments of step c (LDS, or the CIN outer product), FM sums / first-order weights, split
      auto prep = [&](const float* cur, int c) {
        f32x4 a0[MT], a1[MT];
        if constexpr (A_LDS) {
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const int o = arow[i] * 16 + swz_slot(arow[i], g) * 4;
            a0[i] = *reinterpret_cast<const f32x4*>(cur + o);
            a1[i] = *reinterpret_cast<const f32x4*>(cur + BM * 16 + o);
          }
          if constexpr (FMS)
#pragma unroll
            for (int i = 0; i < MT; ++i) fm_accum(a0[i], a1[i], fm_s[i], fm_q[i]);
          if constexpr (WRING) wsum(c);
        } else {
          if (c == 0) {
            cin_x0(0, x0q[0], kq[0]);
            cin_x0(1, x0q[1], kq[1]);
          }
          cin_a_x(0, 2 * c, x0q[0], kq[0], a0);
          cin_a_x(1, 2 * c + 1, x0q[1], kq[1], a1);
          cin_x0(2 * c + 2, x0q[0], kq[0]);
          cin_x0(2 * c + 3, x0q[1], kq[1]);
        }
#pragma unroll
        for (int i = 0; i < MT; ++i) split3(a0[i], a1[i], ah[i], am[i], al[i]);
      };
      // the six split MFMAs of column tiles [t0, t1) (compile-time after inlining) from the B
      // planes of stage buffer `buf`; dma(q) for q < ndma rides one per tile
      auto tiles = [&](const float* buf, auto T0, auto T1, auto ND, auto&& dma) {
        constexpr int t0 = decltype(T0)::value, t1 = decltype(T1)::value, ndma = decltype(ND)::value;
        const float* Bt = buf + AROWS * 16;
        auto ldb = [&](int t, f32x4* b) {
          const int row = (bt0 + t) * 16 + r16;
          const int o = row * 16 + swz_slot(row, g) * 4;
          b[0] = *reinterpret_cast<const f32x4*>(Bt + o);
          b[1] = *reinterpret_cast<const f32x4*>(Bt + BN * 16 + o);
          b[2] = *reinterpret_cast<const f32x4*>(Bt + 2 * BN * 16 + o);
        };
        constexpr int PF = RMX_STAG_PF;
        f32x4 bq[PF + 1][3];
#pragma unroll
        for (int t = 0; t < NTW; ++t)
          if (t >= t0 && t < t0 + PF && t < t1) ldb(t, bq[(t - t0) % (PF + 1)]);
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
          if (t < t0 || t >= t1) continue;
          if (t + PF < t1 && !RMX_DIAG_NOB) ldb(t + PF, bq[(t - t0 + PF) % (PF + 1)]);
          if (t - t0 < ndma) dma(t - t0);
          __builtin_amdgcn_sched_barrier(0);
          const f32x4* b = bq[(t - t0) % (PF + 1)];
          const bf16x8 bh = __builtin_bit_cast(bf16x8, b[0]);
          const bf16x8 bm = __builtin_bit_cast(bf16x8, b[1]);
          const bf16x8 bl = __builtin_bit_cast(bf16x8, b[2]);
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            f32x4 d = acc[i][t];
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bm, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bh, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bm, d, 0, 0, 0);
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, d, 0, 0, 0);
          }
        }
#pragma unroll
        for (int q = 0; q < NTW; ++q)
          if (q >= t1 - t0 && q < ndma) dma(q);
      };
      // the two halves run separate copies of the loop (LATE is a compile-time flag), so the
      // register allocator sees one straight schedule per copy
      auto run = [&](auto LATE) {
        constexpr bool kLate = decltype(LATE)::value != 0;
        for (int c = 0; c < nchunks; ++c) {
          // bar0(c): this wave's DMAs (A / w / ids of step c by phase 1 of step c - 1, B of step c
          // by phase 2) have landed; after the barrier, every wave's have
          RMX_TMARK(6);  // (diagnostic phases of the staggered loop: 6 tail of phase 2 + this wait)
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          RMX_TMARK(0);  // 0: DMA / LDS wait before bar0
          __builtin_amdgcn_s_barrier();
          RMX_TMARK(1);  // 1: bar0
          const float* cur = smem + (c & 1) * STAGE;
          if constexpr (!kLate) {
            prep(cur, c);
            RMX_TMARK(2);  // 2: prep (X)
            tiles(cur, IC<0>{}, IC<NT1>{}, IC<NP1>{}, [&](int q) { dma1(c, q); });
            RMX_TMARK(3);  // 3: phase-1 tiles
            __builtin_amdgcn_s_barrier();  // bar1(c): Y has read the B planes of step c - 1
            RMX_TMARK(4);  // 4: bar1
            tiles(cur, IC<NT1>{}, IC<NTW>{}, IC<NP2>{}, [&](int q) { dma2(c, q); });
            RMX_TMARK(5);  // 5: phase-2 tiles
          } else {
            if (c > 0) {
              tiles(smem + ((c - 1) & 1) * STAGE, IC<NT1>{}, IC<NTW>{}, IC<NP1>{}, [&](int q) { dma1(c, q); });
            } else {
#pragma unroll
              for (int q = 0; q < NP1; ++q) dma1(c, q);
            }
            RMX_TMARK(3);  // 3: phase-1 tiles
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // its B reads of step c - 1 are done
            __builtin_amdgcn_s_barrier();                        // bar1(c)
            RMX_TMARK(4);  // 4: bar1
            prep(cur, c);
            RMX_TMARK(2);  // 2: prep (Y)
            tiles(cur, IC<0>{}, IC<NT1>{}, IC<NP2>{}, [&](int q) { dma2(c, q); });
            RMX_TMARK(5);  // 5: phase-2 tiles
          }
        }
        if constexpr (kLate)
          if (nchunks > 0) tiles(smem + ((nchunks - 1) & 1) * STAGE, IC<NT1>{}, IC<NTW>{}, IC<0>{}, [&](int) {});
      };
      if (late)
        run(IC<1>{});
      else
        run(IC<0>{});
    } else
    for (int c = 0; c < nchunks; ++c) {
      // (fast rings issue every step's DMAs, past the end too: always RING - 2 younger stages)
      const int younger = (FAST || RING - 2 < nchunks - 1 - c) ? RING - 2 : nchunks - 1 - c;
      RMX_TMARK(6);  // 6: MFMA issue tail of the previous step (+ prologue)
      vm_wait(younger * my_n);                             // this wave's DMAs of chunk c have landed
      RMX_TMARK(0);  // 0: DMA wait
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // and its reads of chunk c - 1 are done
      if constexpr (!(RMX_GEMM_DIAG & 2)) __builtin_amdgcn_s_barrier();  // ... for every wave
      RMX_TMARK(1);  // 1: barrier
      const int cn = c + RING - 1;  // the stage refilled into the buffer of chunk c - 1
      RMX_TMARK(2);
      compute_chunk(smem + (c % RING) * STAGE, 0, c, [&](int q) {
        if (q < kQID) {
          // ids of step c + 2 into the slot of step c (its last reader, the issue of stage c,
          // ran before this step's barrier); past the last step every id is -1 (fields >= F)
          if constexpr (IDRING) {
            if constexpr (S3)
              issue_id(c + 2, q);
            else if (c + 2 < nchunks)
              issue_id(c + 2, q);
          }
        } else if (q < kQID + kQW) {
          // weights of stage c + 1 into the w slot of step c - 1 (read before this step's barrier)
          if constexpr (WRING) {
            if constexpr (S3) {
              issue_w(cn, q - kQID, [&] { return pend_id; });
            } else if (wfuse && cn < nchunks) {
              issue_w(cn, q - kQID, [&] { return w_id(cn, q - kQID); });
            }
          }
        } else if constexpr (FAST) {
          // past the last step: re-read the last step's sources into the free slot (never read)
          issue_s3(cn < nchunks ? cn : nchunks - 1, cn % RING, q - kQID - kQW, [&] { return pend_id; });
        } else if (cn < nchunks) {
          issue_one(cn, q - kQID - kQW);
        }
      }, [&](int q) {
        if constexpr (S3 && WRING) {
          if (q >= kQID && q < kQID + kQW) pend_id = w_id(cn, q - kQID);
        }
        if constexpr (S3 && IDRING) {
          constexpr int QA_ = AINS_ / NW;
          if (q >= kQID + kQW && q < kQID + kQW + QA_) pend_id = a_id(cn < nchunks ? cn : nchunks - 1, q - kQID - kQW);
        }
      });
    }
    RMX_TMARK(6);
#if RMX_GEMM_DIAG & 8
    if (dmark && lane == 0 && (nchunks > 100 || (RMX_GEMM_DIAG & (64 | 128)))) {  // (DIAG & 16: CIN layers 2+)
      for (int k = 0; k < 7; ++k) g_rmx_diag_t[(wid ? 8 : 0) + k] = dsum[k];
      g_rmx_diag_t[(wid ? 8 : 0) + 7] = nchunks;
      if (wid == 0) {
        g_rmx_diag_t[16] = __builtin_amdgcn_s_memtime() - dt0;
        g_rmx_diag_t[17] = __builtin_amdgcn_s_memrealtime() - drt0;
      }
    }
#endif
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // C/D layout of 16x16 MFMA: lane holds rows 4*(lane>>4) + r (r = 0..3), column lane & 15.
  // Stored activations go through LDS (each wave transposes its rows into a private slab of the
  // now idle stage buffers) so the global stores are whole-row float4s instead of 4-B scatters.
  auto store_rows = [&](float* dst, int ldd) {
    if constexpr ((RMX_GEMM_DIAG & 512) != 0) return;  // diagnostic: no epilogue transpose, no stores
    using EG = EpiGeom<T, STAGE>;
    constexpr int RW = EG::RW, NTH = EG::NTH, LD = EG::LD;
    float* wbuf = smem + wid * RW * LD;
#pragma unroll
    for (int j0 = 0; j0 < NTW; j0 += NTH) {
#pragma unroll
      for (int t = 0; t < NTH; ++t) {
        if (j0 + t >= NTW) break;
        const float bn = p.bias ? p.bias[n0 + (bt0 + j0 + t) * 16 + r16] : 0.f;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[i][j0 + t][r] + bn;
            wbuf[(i * 16 + g * 4 + r) * LD + t * 16 + r16] = (p.raw || v > 0.f) ? v : 0.f;
          }
      }
      __syncthreads();
      const int nf4 = ((NTW - j0 < NTH) ? (NTW - j0) : NTH) * 4;
      for (int q = lane; q < RW * nf4; q += 64) {
        const int rr = q / nf4, c4 = q - rr * nf4;
        const int m = m0 + wm * RW + rr;
        if (m < M && !(RMX_GEMM_DIAG & 32)) {
          f32x4 v = *reinterpret_cast<const f32x4*>(wbuf + rr * LD + c4 * 4);
          const int64_t o = (int64_t)m * ldd + n0 + (bt0 + j0) * 16 + c4 * 4;
          if (p.mask) {
            const f32x4 h = *reinterpret_cast<const f32x4*>(p.mask + (int64_t)m * p.ldmask + n0 + (bt0 + j0) * 16 + c4 * 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = h[e] > 0.f ? v[e] : 0.f;
          }
          if constexpr (!BF) {
            if (p.eg_x) {
              const int n = n0 + (bt0 + j0) * 16 + c4 * 4;
              const f32x4 xv = *reinterpret_cast<const f32x4*>(p.eg_x + (int64_t)m * p.eg_ldx + n);
              const f32x4 sv = *reinterpret_cast<const f32x4*>(p.eg_s + (int64_t)m * 16 + (n & 15));
              const float gz = p.eg_dz[m];
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += gz * (sv[e] - xv[e]) / 16.0f;
            }
          }
          if constexpr (BF)
            *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(dst) + o) = __builtin_convertvector(v, bf16x4);
          else if (p.nt_store)
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst + o));
          else
            *reinterpret_cast<f32x4*>(dst + o) = v;
        }
      }
      __syncthreads();
    }
  };
  if constexpr (FM) {
    if (fm_on) {
      // y2 = 0.5 * (sum_j (s_j^2 - q_j) / k), j sequential over the four lane groups; y1 = sum_f w in
      // field order (encoder_k16_kernel<1> arithmetic); one lane per row writes y1 + y2
#pragma clang fp contract(off)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        float a = 0.f;
        if constexpr (FMS) {
          if (fm_sums) {
            float d[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) d[t] = fm_s[i][t] * fm_s[i][t] - fm_q[i][t];
#pragma unroll
            for (int gg = 0; gg < 4; ++gg)
#pragma unroll
              for (int t = 0; t < 4; ++t) a += __shfl(d[t], gg * 16 + r16);
          }
        }
        // y1: lane group g loads the weights of fields g, g + 4, ...; they are summed in field order
        // (loading them before the main loop measured slower: it holds 10 more registers through it)
        const int m = m0 + arow[i];
        if (p.fm_add) {
          if (g == 0 && wn == 0 && m < M) p.fm_y[m] = p.fm_y[m] + 0.5f * (a / 16.0f);
          continue;
        }
        if constexpr (WRING) {
          if (wfuse) {  // y1 summed per K step from the w ring
            if (g == 0 && wn == 0 && m < M) p.fm_y[m] = fm_sums ? y1acc[i] + 0.5f * (a / 16.0f) : y1acc[i];
            continue;
          }
        }
        float wv[kFmMaxF / 4];
#pragma unroll
        for (int u = 0; u < kFmMaxF / 4; ++u) {
          const int f = u * 4 + g;
          int id = 0;
          if (f < F) {
            if constexpr (IDRING) id = p.ga.ids[(int64_t)(m0 + arow[i] < M ? m0 + arow[i] : m0) * F + f];
            else id = sids[arow[i] * F + f];
          }
          wv[u] = f < F ? (p.fm_w_bf16 ? (float)reinterpret_cast<const bf16_t*>(p.fm_w)[(int64_t)id << p.fm_wsh]
                                       : reinterpret_cast<const float*>(p.fm_w)[(int64_t)id << p.fm_wsh])
                        : 0.f;
        }
        float y1 = 0.f;
#pragma unroll
        for (int f = 0; f < kFmMaxF; ++f)
          if (f < F) y1 += __shfl(wv[f >> 2], (f & 3) * 16 + r16);
        if (g == 0 && wn == 0 && m < M) p.fm_y[m] = fm_sums ? y1 + 0.5f * (a / 16.0f) : y1;
      }
    }
  }
  if constexpr (EPI == kEpiRelu) {
    if (p.xcol) {  // DCN: the cross dot products ride along as extra raw columns
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int e = n0 + (bt0 + j) * 16 + r16 - p.xn_main;
          if (e >= 0 && e < p.xld)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int m = m0 + wm * MT * 16 + i * 16 + g * 4 + r;
              if (m < M) p.xcol[(int64_t)m * p.xld + e] = acc[i][j][r];
            }
        }
    }
    store_rows(p.C, p.ldc);
  } else {
    // row reduction sum_n ReLU(acc + b)[n] * w[n] over the block's (= the layer's) columns;
    // with WN > 1 the waves of a row group add their partial sums through LDS
    float* red = smem;  // [WN][BM], the stage buffers are idle after the last barrier
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int rl = wm * MT * 16 + i * 16 + g * 4;  // block-local first row of the lane group
      float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int n = n0 + (bt0 + j) * 16 + r16;
        const float bn = p.bias[n];
        const float wv = EPI == kEpiOutput ? p.oa.wo[n] : p.wo[n];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bn;
          v = v > 0.f ? v : 0.f;
          part[r] += v * wv;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = part[r];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        part[r] = v;
      }
      if (r16 < 4) {
        const float y = r16 == 0 ? part[0] : (r16 == 1 ? part[1] : (r16 == 2 ? part[2] : part[3]));
        red[wn * BM + rl + r16] = y;
      }
    }
    __syncthreads();
    for (int rl = tid; rl < BM; rl += NTHR) {
      const int m = m0 + rl;
      if (m >= M) continue;
      float y = red[rl];
#pragma unroll
      for (int w = 1; w < WN; ++w) y += red[w * BM + rl];
      if constexpr (EPI == kEpiCin) {
        p.rowdot[m] = p.cin_first ? y : p.rowdot[m] + y;
      } else {
        const OutArgs& oa = p.oa;
        if (gridDim.y > 1) {  // a column slice of the layer: partial logit, out_finish_kernel combines
          oa.part[(int64_t)by * M + m] = y;
          continue;
        }
        if (oa.has_bo) y = y + oa.bo;
        if (oa.rowsum) {
          float rs = 0.f;
          for (int jj = 0; jj < oa.rowsum_k; ++jj) rs += oa.rowsum[(int64_t)m * oa.rowsum_k + jj];
          y = rs + y;
        }
        if (oa.pre2) y = oa.pre2[m] + y;
        float t = oa.pre ? oa.pre[m] + y : y;
        t = t + oa.beta;
        oa.out[m] = 1.0f / (1.0f + expf(-t));
      }
    }
    if constexpr (EPI == kEpiCin) {
      if (p.C) {
        __syncthreads();  // red[] lives in the slab area
        store_rows(p.C, p.ldc);  // u_l for the next CIN layer
      }
    }
  }
#if RMX_GEMM_DIAG & 256
  if (kDiagSel && threadIdx.x == 0) {
    const int bid = blockIdx.y * gridDim.x + blockIdx.x;
    if (bid < 4096) {
      g_rmx_blk[bid][0] = blk_t0;
      g_rmx_blk[bid][1] = __builtin_amdgcn_s_memrealtime();
      g_rmx_blk[bid][2] = __smid() | ((unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 16);  // | XCC_ID << 16
    }
  }
#endif
}


// -------------------------------------------------------------- dispatch ----

// column tiles per block that have kernels (a layer's Npad is a multiple of one of them)
constexpr int kNTs[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 13, 16, 20, 25, 26};
constexpr int kCinNTs[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 13, 16};

template <class T, int AMODE, int EPI, int PREC = kPrecF32>
int launch_cfg(hipStream_t s, GemmArgs& p) {
  using SG = StageGeom<T, AMODE, PREC>;
  size_t lds = sizeof(float) * T::NBUF * SG::FLOATS;
  if (kIdRing<T, AMODE, PREC>) {
    if (!p.ga.ids) {
      set_error("gemm: the id-ring gather needs an explicit id array");
      return RMX_E_INVALID;
    }
    lds += sizeof(int) * 8 * T::BM;  // id ring + first-order weight ring
  } else if (AMODE == kGatherK16 || AMODE == kGatherAny) {
    lds += sizeof(int) * T::BM * p.ga.F;
    if (kWRing<T, AMODE, PREC> && EPI == kEpiRelu) lds += sizeof(float) * 4 * T::BM;  // first-order weight ring
  }
  if (AMODE == kCinOuter) lds += sizeof(float) * T::BM * p.XS + (p.cmap ? sizeof(int) * p.ncmap : 0);
  if (p.cmap && (AMODE != kCinOuter || PREC != kPrecS3)) {
    set_error("gemm: a CIN chunk map needs the split CIN kernel");
    return RMX_E_INVALID;
  }
  if (EPI != kEpiOutput) lds = std::max(lds, sizeof(float) * EpiGeom<T, SG::FLOATS>::FLOATS);
  lds = std::max(lds, sizeof(float) * T::WN * T::BM);  // row-reduction partials
  if (lds > 160 * 1024) {
    set_error("gemm: LDS budget exceeded (" + std::to_string(lds) + " bytes)");
    return RMX_E_INVALID;
  }
  if (p.Npad % T::BN) {
    set_error("gemm: Npad " + std::to_string(p.Npad) + " is not a multiple of the block width");
    return RMX_E_INVALID;
  }
  if (T::RING > 0 && AMODE == kDenseA && (int64_t)p.M * p.lda >= (int64_t)1 << 32) {
    set_error("gemm: batch too large for one launch (M * lda >= 2^32 elements)");
    return RMX_E_INVALID;
  }
  if (EPI == kEpiCin && p.Npad != T::BN) {
    set_error("gemm: a CIN layer must fit one block");
    return RMX_E_INVALID;
  }
  if (EPI == kEpiOutput && p.Npad != T::BN && !p.oa.part) {
    set_error("gemm: a sliced output layer needs the partial-logit buffer");
    return RMX_E_INVALID;
  }
  dim3 grid((p.M + T::BM - 1) / T::BM, p.Npad / T::BN);
  auto kern = gemm_kernel<T, AMODE, EPI, PREC>;
  if (lds > 64 * 1024)
    RMX_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, grid, dim3(T::NTHR), lds, s, p);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

template <class T, int PREC>
int launch_epi(hipStream_t s, GemmArgs& p, int amode, Epi epi) {
#define RMX_EPI(AM)                                                            \
  if (epi == Epi::kReluStore) return launch_cfg<T, AM, kEpiRelu, PREC>(s, p); \
  return launch_cfg<T, AM, kEpiOutput, PREC>(s, p);
  if (amode == kDenseA) { RMX_EPI(kDenseA) }
  if (amode == kGatherK16) { RMX_EPI(kGatherK16) }
  RMX_EPI(kGatherAny)
#undef RMX_EPI
}

// the tower_variant launch_tower_nt uses at M >= 65536 (knob, else the default below)
inline int tower_variant_for(int NT, Epi epi, bool bf16, int K) {
  const bool even = NT % 2 == 0 && NT >= 8;
  // (bf16 K >= 1024, PNN layer 1: variant 6, 0.089-0.091 vs 0.093-0.094 ms for variant 3 at B = 65,536,
  // profiles/r05/ab_bf16_variant.txt)
  const int def = NT == 26 ? ((epi == Epi::kOutput && !bf16) ? 5 : (bf16 && K >= 1024 ? 6 : 4)) : (even ? 3 : 0);
  return tuning_get("tower_variant", def);
}

// a bf16 tower layer of Npad columns runs in 208-column slices (tower variant 6): an output layer
// then writes partial logits and out_finish_kernel combines them
inline bool bf16_tower_sliced(int Npad, Epi epi, int K, int M, int amode) {
  return Npad == 416 && M >= 65536 && amode != kGatherAny && tower_variant_for(26, epi, true, K) == 6;
}

template <int NT, int PREC>
int launch_tower_nt(hipStream_t s, GemmArgs& p, int amode, Epi epi) {
  // Large batches (M >= 65536, >= 2 blocks of 128 rows per CU).  Knob "tower_variant":
  //   0: register-staged double buffer, 8 waves on M x all NT tiles per wave (2 waves / SIMD);
  //   1: LDS-DMA ring (4 chunks), same tiling;
  //   2: LDS-DMA ring (3 chunks), 4 x 2 waves of 32 rows x NT/2 tiles;
  //   3: LDS-DMA ring (3 chunks), 8 x 2 waves of 16 rows x NT/2 tiles, 4 waves / SIMD in one
  //      16-wave block (default for even NT >= 8 other than 26): N = 400, M = 65536, fp32
  //      0.289 ms/layer vs 0.315 (variant 0); bf16 0.063 vs 0.092;
  //   4: LDS-DMA ring (2 chunks), 4 x 2 waves of 16 rows, 2 blocks / CU (NT = 26);
  //   5: LDS-DMA ring (2 chunks), 4 x 2 waves of 32 rows, 2 blocks / CU (NT = 26).
  // Variants 2 / 3 need an even NT.  Small batches: 4-wave blocks, register-staged.
  constexpr bool kEven = NT % 2 == 0 && NT >= 8;
  // defaults (A/B'd with tools/tune.py, N = 400 padded to 26 tiles): 8-wave blocks with a 2-deep
  // LDS-DMA ring fit 2 blocks per CU (one block's epilogue overlaps the other's MFMAs): fp32
  // 0.280 / 0.183 ms for layers 1 / 2 vs 0.288 / 0.189 (variant 3), bf16 DCN 457 vs 431 M ex/s; the
  // fp32 output layer prefers 32 rows per wave (variant 5: 0.171 vs 0.177 ms)
  // bf16 layers with a long K (PNN layer 1: K = 624 + 741) prefer the 3-deep rings: the 16-wave one
  // (variant 3: 0.098 vs 0.119 ms at B = 65,536) and, since round 5, the fast ring tile (variant 6)
  int var = tower_variant_for(NT, epi, PREC == kPrecBF16, p.K);
  if (p.M >= 65536) {
    if constexpr (kEven) {
      if (var == 2) return launch_epi<Tile<2, NT / 2, 4, 2, 1, 1, 3>, PREC>(s, p, amode, epi);
      if (var == 3) return launch_epi<Tile<1, NT / 2, 8, 2, 1, 4, 3>, PREC>(s, p, amode, epi);
      if constexpr (NT == 26) {
        if (var == 4) return launch_epi<Tile<1, NT / 2, 4, 2, 1, 4, 2>, PREC>(s, p, amode, epi);
        if (var == 5) return launch_epi<Tile<2, NT / 2, 4, 2, 1, 2, 2>, PREC>(s, p, amode, epi);
        // 6 (bf16): the fast ring tile -- 8 waves of 32 rows x 208 columns (two column slices,
        // XCD-paired), 3-deep branch-free LDS-DMA ring, 1 block / CU
        if constexpr (PREC == kPrecBF16)
          if (var == 6 && amode != kGatherAny) return launch_epi<Tile<2, NT / 2, 8, 1, 1, 2, 3, 0, 1>, PREC>(s, p, amode, epi);
      }
    }
    if (var == 1) return launch_epi<Tile<1, NT, 8, 1, 1, 1, 4>, PREC>(s, p, amode, epi);
    if (amode == kDenseA) return launch_epi<Tile<1, NT, 8, 1, 2, 1>, PREC>(s, p, amode, epi);
    return launch_epi<Tile<1, NT, 8, 1, 1, 1>, PREC>(s, p, amode, epi);
  }
  return launch_epi<Tile<1, NT, 4, 1, 1, 1>, PREC>(s, p, amode, epi);
}

template <int NT>
int launch_cin_nt(hipStream_t s, GemmArgs& p) {
  // knob "cin_variant": 0 = 8 waves x 16 rows, 2 chunks per stage, 4 waves / SIMD (two blocks
  // per CU: 1.637 ms / layer at B = 4,096 vs 1.84 at 3 waves / SIMD); 1 = 8 waves x 32 rows.
  // Small M always uses 4 waves x 16 rows.  (An LDS-DMA ring for the weight chunks measured 4-8 %
  // slower: the A operand is built in registers, so the register-staged W stage is cheap.)
  const int var = tuning_get("cin_variant", 0);
  if (p.M < 8192) return launch_cfg<Tile<1, NT, 4, 1, 2, 1>, kCinOuter, kEpiCin>(s, p);
  if (var == 1) return launch_cfg<Tile<2, NT, 8, 1, 2, 1>, kCinOuter, kEpiCin>(s, p);
  return launch_cfg<Tile<1, NT, 8, 1, 2, 4>, kCinOuter, kEpiCin>(s, p);
}


int launch_tower_bf16(hipStream_t s, GemmArgs& p, int nt, int amode, Epi epi);
// kPrecS3 (k_gemm_s3.hip): tower layers with Npad % 208 == 0, CIN layers with Npad == 208
constexpr int kS3BN = 208;
int launch_tower_s3(hipStream_t s, GemmArgs& p, int amode, Epi epi);
int launch_cin_s3(hipStream_t s, GemmArgs& p);

}  // namespace rmx
