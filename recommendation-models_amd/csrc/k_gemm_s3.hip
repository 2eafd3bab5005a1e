// k_gemm_s3.hip -- fp32 tower / CIN GEMMs on the bf16 matrix cores through an exact 3-way split
// (k_gemm.hpp kPrecS3), gfx950.
//
// Why: on gfx950 v_mfma_f32_16x16x4_f32 runs at 64 FLOP/clk/SIMD (157 TF), 1/16 of
// v_mfma_f32_16x16x32_bf16.  Every normal fp32 x is exactly hi + mid + lo with three bf16 parts
// (8 significand bits each), so x*y = sum of 9 exact bf16 products; the six kept ones
// (hi*hi, hi*mid, mid*hi, hi*lo, lo*hi, mid*mid) leave out mid*lo + lo*mid + lo*lo <=
// (2^-24 + 2^-34) |x y| (|mid| <= 2^-8 |x|, |lo| <= 2^-17 |x|): the size of one rounding of the
// fp32 FMA chain the reference's MKL sgemm (and our f32 MFMA path) performs per product.
// Six bf16 MFMAs cost 96 cycles per 16x16x32 tile step against 256 for eight f32 MFMAs.
// Parity is checked against the fp64 oracle at the same 1e-5 bar as the f32 path
// (tests/test_gpu_parity.py, test_split_gemm.py); rmx_set_tuning("f32_split", 0) selects the
// f32 MFMA engine.
//
// The semantics are those of k_gemm.hip (HigherOrderEncoder.scala:34-59 tower layers,
// CINEncoder.scala:36-58 / 105-176 CIN layers); only the arithmetic of the K reduction differs.
#include "k_gemm.hpp"

namespace rmx {

bool f32_split_enabled() { return tuning_get("f32_split", 1) != 0; }

int64_t split3_elems(int n16, int Npad) { return (int64_t)((n16 + 1) / 2) * 3 * Npad * 32; }

// fp32 packed [n16][Npad][16] -> [steps][3][Npad][32] bf16 (steps = ceil(n16 / 2)).  Position
// 8g + 4h + q of a 32-wide step holds element 4g + q of fp32 chunk 2s + h: the K order in which
// lane group g of the split A fragment holds its values (k_gemm.hpp compute_step_s3).
__global__ void pack_split3_kernel(const float* __restrict__ Wp, int n16, int Npad, int64_t tot,
                                   bf16_t* __restrict__ W3) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int pos = (int)(i & 31);
  const int64_t rest = i >> 5;
  const int n = (int)(rest % Npad);
  const int64_t s = rest / Npad;
  const int g = pos >> 3, h = (pos >> 2) & 1, q = pos & 3;
  const int64_t c = 2 * s + h;
  const float v = c < n16 ? Wp[(c * Npad + n) * 16 + 4 * g + q] : 0.f;
  const bf16_t hi = (bf16_t)v;
  const float r = v - (float)hi;
  const bf16_t mid = (bf16_t)r;
  const bf16_t lo = (bf16_t)(r - (float)mid);
  const int64_t plane = (int64_t)Npad * 32;
  const int64_t o = s * 3 * plane + (int64_t)n * 32 + pos;
  W3[o] = hi;
  W3[o + plane] = mid;
  W3[o + 2 * plane] = lo;
}

int launch_pack_split3(hipStream_t s, const float* Wp, int n16, int Npad, bf16_t* W3) {
  const int64_t tot = (int64_t)((n16 + 1) / 2) * Npad * 32;
  if (tot <= 0) return RMX_OK;
  hipLaunchKernelGGL(pack_split3_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, Wp, n16, Npad, tot,
                     W3);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// W^T of a Linear(in = K, out = N) at L.w_off (single block, no extra rows): element (col j, k n) =
// W[n][j], packed [KTpad/16][NTpad][16] fp32
__global__ void pack_linear_t_kernel(const float* __restrict__ mats, int64_t w_off, int N, int K, int KTpad,
                                     int NTpad, float* __restrict__ Wp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)KTpad * NTpad) return;
  const int kk = (int)(i & 15);
  const int64_t rest = i >> 4;
  const int j = (int)(rest % NTpad);
  const int n = (int)(rest / NTpad) * 16 + kk;
  Wp[i] = (n < N && j < K) ? mats[w_off + (int64_t)n * K + j] : 0.f;
}

int launch_pack_linear_t(hipStream_t s, const float* mats_dev, DenseLayer& L) {
  if (!L.WT) return RMX_OK;
  const int64_t tot = (int64_t)L.KTpad * L.NTpad;
  hipLaunchKernelGGL(pack_linear_t_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, mats_dev, L.w_off,
                     L.N, L.K, L.KTpad, L.NTpad, L.WT);
  RMX_HIP(hipGetLastError());
  return launch_pack_split3(s, L.WT, L.KTpad / 16, L.NTpad, L.WT3);
}

// C_l^T of a CIN layer (C_l: H x F*Hp at c.w_off) packed like a Linear's W^T: element (col j, k h) =
// C_l[h][j], [KTpad/16][NTpad][16], then split into the three bf16 planes
int launch_pack_cin_t(hipStream_t s, const float* mats_dev, int F, CinLayer& c) {
  const int64_t tot = (int64_t)c.KTpad * c.NTpad;
  hipLaunchKernelGGL(pack_linear_t_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, mats_dev, c.w_off,
                     c.H, F * c.Hp, c.KTpad, c.NTpad, c.WT);
  RMX_HIP(hipGetLastError());
  return launch_pack_split3(s, c.WT, c.KTpad / 16, c.NTpad, c.WT3);
}

// dz[r][j] = sum_h gpre[r][h] C_l[h][j] for rows r of a chunk, on the split GEMM (raw store, no bias);
// dz has row stride ldz >= c.NTpad (columns past F*Hp come out zero)
int launch_cin_dz_s3(hipStream_t s, const CinLayer& c, int rows, const float* gpre, int ldg, float* dz, int ldz) {
  if (!c.WT3 || ldz < c.NTpad) {
    set_error("cin backward: no split-GEMM C^T planes for this layer");
    return RMX_E_INVALID;
  }
  if (rows <= 0) return RMX_OK;
  GemmArgs p{};
  p.M = rows;
  p.K = c.H;
  p.Kpad = (c.KTpad / 16 + 1) / 2 * 32;
  p.Npad = c.NTpad;
  p.A = gpre;
  p.lda = ldg;
  p.Wp = reinterpret_cast<const float*>(c.WT3);
  p.bias = nullptr;
  p.C = dz;
  p.ldc = ldz;
  p.raw = 1;
  return launch_tower_s3(s, p, kDenseA, Epi::kReluStore);
}

bool dx_s3_usable(const DenseLayer& L, int ldx) {
  return L.WT3 && f32_split_enabled() && L.NTpad % kS3BN == 0 && L.NTpad <= ldx;
}

int launch_dx_s3(hipStream_t s, const DenseLayer& L, int B, const float* dpre, int lda, float* dx, int ldx,
                 const float* mask, int ldmask, const EmbGradArgs* eg) {
  if (!dx_s3_usable(L, ldx) || (mask && L.NTpad > ldmask)) {
    set_error("dx: no split-GEMM W^T for this layer");
    return RMX_E_INVALID;
  }
  if (B <= 0) return RMX_OK;
  GemmArgs p{};
  p.M = B;
  p.K = L.N;
  p.Kpad = (L.KTpad / 16 + 1) / 2 * 32;
  p.Npad = L.NTpad;
  p.A = dpre;
  p.lda = lda;
  p.Wp = reinterpret_cast<const float*>(L.WT3);
  p.bias = nullptr;
  p.C = dx;
  p.ldc = ldx;
  p.raw = 1;
  p.mask = mask;
  p.ldmask = ldmask;
  if (eg) {
    if (ldx != L.K || L.K % 16 || ldx % 4 || eg->ldx % 4) {
      set_error("dx: the fused embedding gradient needs [B][F * 16] rows");
      return RMX_E_INVALID;
    }
    p.eg_x = eg->x;
    p.eg_s = eg->s;
    p.eg_dz = eg->dz;
    p.eg_ldx = eg->ldx;
  }
  return launch_tower_s3(s, p, kDenseA, Epi::kReluStore);
}

// Output head of a layer computed in ny column slices: logit = sum of the slices' partial dots
// (slice order), then the same combination as the fused epilogue (k_gemm.hpp kEpiOutput).
__global__ __launch_bounds__(256) void out_finish_kernel(int M, int ny, OutArgs oa) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float y = oa.part[m];
  for (int j = 1; j < ny; ++j) y += oa.part[(int64_t)j * M + m];
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

int launch_out_finish(hipStream_t s, int M, int ny, const OutArgs& oa) {
  if (M <= 0) return RMX_OK;
  hipLaunchKernelGGL(out_finish_kernel, dim3((M + 255) / 256), dim3(256), 0, s, M, ny, oa);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// Tower layer, kPrecS3.  Blocks of 8 waves x 16 (or 32) rows span 208 columns (13 tiles), so a
// 400-wide layer (Npad 416) runs as 2 column slices; one K step = 32 (A: two fp32 chunks, B: the
// three bf16 planes) through a 2-deep LDS-DMA ring.  Knob "s3_tower":
//   0  MT = 1: 56 KiB per stage (128 A rows x 2 + 208 x 3 B rows), 1 block / CU;
//   1  MT = 2 (BM = 256, 71 KiB per stage; halves the B fragment reads per MFMA) on dense A and on
//      k = 16 gathers with an id array (ids by DMA into a 4 KiB LDS ring: a [BM][F] id tile would
//      not fit; streaming them through registers measured slower and spilled) -- the default: DeepFM 400^3 at
//      B = 65,536, layers 2 / 3: 0.125 / 0.117 ms vs 0.136 / 0.128 (MT = 1) and 0.194 / 0.174
//      on the f32 MFMA engine;
//   2  MT = 1, register-staged double buffer.
constexpr int kS3NT = 13;

// the 32-row tile (MT = 2): on dense A and on k = 16 gathers with an id array, while its blocks
// still cover every CU (M = 16,384 x 400: 128 blocks of 256 rows ran 0.055 ms vs 0.038 with 256
// blocks of 128 rows)
static bool s3_mt2(int M, int Npad, int amode, bool ids) {
  const int64_t blocks2 = (int64_t)(M + 255) / 256 * (Npad / (kS3NT * 16));
  return tuning_get("s3_tower", 1) == 1 && (amode == kDenseA || (amode == kGatherK16 && ids)) && blocks2 >= 256;
}

int launch_tower_s3(hipStream_t s, GemmArgs& p, int amode, Epi epi) {
  if (p.fm_w && p.fm_w_bf16) {
    set_error("split GEMM: fp32 layers take an fp32 table");
    return RMX_E_INVALID;
  }
  const int var = tuning_get("s3_tower", 1);
  p.prio = tuning_get("gemm_prio", 0);
  p.nt_store = tuning_get("gemm_nt_store", 0);
  // p.cols32 (knob "s3_cols", round 6): 128-row x 32-column blocks for small launch batches.  The whole-tower
  // kernel (k_small_s3.hip) streams every layer's split planes through EVERY block (3.67 MB per 16 samples);
  // here each block streams 1/13 of a layer's planes and its 128 A rows come from the materialised x / h in
  // L2 (the 13 column blocks of a row block run on one XCD: blockIdx.x = row block, and the grid's row-block
  // count is a multiple of 8 at the batches that take it).  Same products in the same K order per output.
  if (p.cols32 && amode == kDenseA) {
    // knob "s3_cols_ring" (the 8-wave blocks): LDS-DMA ring depth (2, 3 (default) or 4 stages of 22 KiB).  At B = 1,024 the
    // layers took 0.0206 / 0.0153 / 0.0193 ms on 2 stages, 0.0168 / 0.0130 / 0.0172 on 3, 0.0166 / 0.0128 /
    // 0.0169 on 4; 4 lost at B >= 4,096 (profiles/r06/ab_cols32.txt)
    const int rg = tuning_get("s3_cols_ring", 3);
    // knob "s3_cols_wm": waves (16 rows each) per block, 4 (default), 8 or 2.  At B = 1,024: 19.2 M examples/s
    // on 8 (104 blocks), 22.9 M on 4 (208 blocks), 20.5 M on 2; at 2,048: 37.7 / 39.2 / 39.0 M
    // (profiles/r06/ab_cols32_wm.txt)
    const int wm = tuning_get("s3_cols_wm", 4);
    if (wm == 4) return launch_epi<Tile<1, 2, 4, 1, 1, 2, 3>, kPrecS3>(s, p, amode, epi);
    if (wm == 2) return launch_epi<Tile<1, 2, 2, 1, 1, 2, 3>, kPrecS3>(s, p, amode, epi);
    if (rg == 2) return launch_epi<Tile<1, 2, 8, 1, 1, 2, 2>, kPrecS3>(s, p, amode, epi);
    if (rg == 3) return launch_epi<Tile<1, 2, 8, 1, 1, 2, 3>, kPrecS3>(s, p, amode, epi);
    return launch_epi<Tile<1, 2, 8, 1, 1, 2, 4>, kPrecS3>(s, p, amode, epi);
  }
  if (var == 2) return launch_epi<Tile<1, kS3NT, 8, 1, 1, 2, 0>, kPrecS3>(s, p, amode, epi);
  // 3: 16-row waves, a single-buffered 57 KiB stage, two blocks per CU (4 waves / SIMD)
  if (var == 3) return launch_epi<Tile<1, kS3NT, 8, 1, 1, 4, 1>, kPrecS3>(s, p, amode, epi);
  // 4: 32-row waves, 4-wave blocks on a single-buffered 55 KiB stage, two blocks per CU (the partner
  // wave on a SIMD belongs to the other block, so one block's DMA wait / epilogue meets the other's MFMAs)
  if (var == 4) return launch_epi<Tile<2, kS3NT, 4, 1, 1, 2, 1>, kPrecS3>(s, p, amode, epi);
  // knob "s3_narrow" (default 1): 2-wave blocks (32 rows x 208 columns) when the 8-wave tile's blocks would
  // leave CUs idle -- small launch batches (B = 4,096: 64 -> 256 blocks).  Same products in the same K
  // order (bitwise).  DeepFM's layers on the engine at B = 4,096: 0.0486 / 0.0288 / 0.0270 ->
  // 0.0444 / 0.0265 / 0.0249 ms (profiles/r04/ab_small_rt.txt)
  if (tuning_get("s3_narrow", 1) != 0 && !s3_mt2(p.M, p.Npad, amode, p.ga.ids != nullptr)) {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
    const int64_t blocks8 = (int64_t)(p.M + 127) / 128 * (p.Npad / (kS3NT * 16));
    if (blocks8 < ncu) return launch_epi<Tile<1, kS3NT, 2, 1, 1, 2, 2>, kPrecS3>(s, p, amode, epi);
  }
  if (s3_mt2(p.M, p.Npad, amode, p.ga.ids != nullptr)) {
    // knob "s3_dense" (dense-A layers at this size; all accumulate in the same K order: equal bits):
    //   5 (default) 16 waves of 16 rows, 4 per SIMD, 2-deep ring (the CIN's s3_cin 4 shape; DeepFM at
    //     B = 65,536: layer 2 0.1075, layer 3 0.0929 ms);
    //   4 stored layers on 4-wave blocks of 32-row waves, two blocks per CU, single-buffered (layer 2
    //     0.1075 vs 0.1114 ms staggered; the gathered layer 1 loses on it, 0.215 vs 0.181: it waits
    //     out every random-row gather);  1 the staggered 8-wave tile (layer 3 0.0959 ms).
    if (amode == kDenseA) {
      const int dv = tuning_get("s3_dense", 5);
      if (dv == 5) return launch_epi<Tile<1, kS3NT, 16, 1, 1, 4, 2>, kPrecS3>(s, p, amode, epi);
      if (dv == 4 && epi == Epi::kReluStore) return launch_epi<Tile<2, kS3NT, 4, 1, 1, 2, 1>, kPrecS3>(s, p, amode, epi);
    }
    // knob "s3_stagger": 1 (default) staggered loop on every tower layer, 2 also on the CIN, 0 off
    // (DeepFM 400^3 at B = 65,536: layers 0.1753 / 0.1110 / 0.0961 ms -> 0.1746 / 0.1082 / 0.0928;
    // the CIN runs slower staggered: 3.06 -> 3.16 ms per layer, its B planes then get half a step
    // of DMA lead)
    if (tuning_get("s3_stagger", 1) != 0)
      return launch_epi<Tile<2, kS3NT, 8, 1, 1, 2, 2, 1>, kPrecS3>(s, p, amode, epi);
    return launch_epi<Tile<2, kS3NT, 8, 1, 1, 2, 2>, kPrecS3>(s, p, amode, epi);
  }
  return launch_epi<Tile<1, kS3NT, 8, 1, 1, 2, 2>, kPrecS3>(s, p, amode, epi);
}

// CIN layer, kPrecS3 (H <= 208): only the B planes go through LDS (39 KiB per K step); the A
// operand x0[f] * u[h] is formed in fp32 registers and split there.  Knob "s3_cin":
//   0  MT = 1, 2-deep LDS-DMA ring;  1  MT = 1, 3-deep ring;  2 (default)  MT = 2, 8 waves, 2-deep
//   ring (CIN 200^3 at B = 16,384, layer 2: 3.73 ms vs 4.60 (MT = 1, 8 waves) and 6.69 on the f32
//   MFMA engine);  3  MT = 1, register-staged double buffer;  4  MT = 1, 16 waves (4 per SIMD), 2-deep
//   ring: twice the B-fragment LDS reads of 2, hidden by the extra waves on some boxes (layers 2+
//   3.022 vs 3.037 ms) but not on others: with the chunk map, 3 boxes gave layers 2+ 3.04-3.07 ms on
//   2 against 3.25-3.27 on 4 (xDeepFM 2.29 -> 2.42 M examples/s).
int launch_cin_s3(hipStream_t s, GemmArgs& p) {
  const int var = tuning_get("s3_cin", 2);
  p.prio = tuning_get("gemm_prio", 0);
  p.nt_store = tuning_get("gemm_nt_store", 0);
  if (var == 1) return launch_cfg<Tile<1, kS3NT, 8, 1, 1, 2, 3>, kCinOuter, kEpiCin, kPrecS3>(s, p);
  if (var == 2) {
    // knob "cin_narrow" (default 1): when the 256-row blocks would leave CUs idle (B * k rows < 256 CUs x
    // 256: xDeepFM below B = 4,096), the largest of 128-, 64- and 32-row blocks that still gives every
    // CU one (MT = 1, 8 / 4 / 2 waves).  Each block then streams all of C_l's planes for fewer rows, but
    // every CU does.  Same products in the same K order (bitwise).  xDeepFM at B = 1,024: CIN layers 2 / 3
    // 0.735 -> 0.301 ms, 0.61 -> 1.38 M examples/s; B = 2,048: 1.21 -> 1.99 M (profiles/r04/ab_cin_narrow.txt)
    if (tuning_get("cin_narrow", 1) != 0 && tuning_get("s3_stagger", 1) != 2) {
      int dev = 0, ncu = 256;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        ncu = 256;
      const int64_t nslice = p.Npad / (kS3NT * 16);
      auto blocks = [&](int rows) { return (int64_t)(p.M + rows - 1) / rows * nslice; };
      if (blocks(256) < ncu) {
        if (blocks(128) >= ncu) return launch_cfg<Tile<1, kS3NT, 8, 1, 1, 2, 2>, kCinOuter, kEpiCin, kPrecS3>(s, p);
        if (blocks(64) >= ncu) return launch_cfg<Tile<1, kS3NT, 4, 1, 1, 2, 2>, kCinOuter, kEpiCin, kPrecS3>(s, p);
        return launch_cfg<Tile<1, kS3NT, 2, 1, 1, 2, 2>, kCinOuter, kEpiCin, kPrecS3>(s, p);
      }
    }
    if (tuning_get("s3_stagger", 1) == 2)
      return launch_cfg<Tile<2, kS3NT, 8, 1, 1, 2, 2, 1>, kCinOuter, kEpiCin, kPrecS3>(s, p);
    return launch_cfg<Tile<2, kS3NT, 8, 1, 1, 2, 2>, kCinOuter, kEpiCin, kPrecS3>(s, p);
  }
  if (var == 3) return launch_cfg<Tile<1, kS3NT, 8, 1, 1, 2, 0>, kCinOuter, kEpiCin, kPrecS3>(s, p);
  if (var == 4) return launch_cfg<Tile<1, kS3NT, 16, 1, 1, 4, 2>, kCinOuter, kEpiCin, kPrecS3>(s, p);
  return launch_cfg<Tile<1, kS3NT, 8, 1, 1, 2, 2>, kCinOuter, kEpiCin, kPrecS3>(s, p);
}

}  // namespace rmx

#if RMX_GEMM_DIAG & 8
// diagnostic builds only: the per-phase cycle sums of the last split-GEMM launch
extern "C" int rmx_diag_phases(unsigned long long* out16) {
  return hipMemcpyFromSymbol(out16, HIP_SYMBOL(rmx::g_rmx_diag_t), sizeof(unsigned long long) * 18) == hipSuccess
             ? 0
             : -5;
}
#endif

#if RMX_GEMM_DIAG & 256
// diagnostic builds only: the per-block timeline of the last selected split-GEMM launch
extern "C" int rmx_diag_blocks(unsigned long long* out, int nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rmx::g_rmx_blk), sizeof(unsigned long long) * 3 * nblocks) == hipSuccess
             ? 0
             : -5;
}
#endif
