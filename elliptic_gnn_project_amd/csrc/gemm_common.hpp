// Shared pieces of the K7 GEMM kernels (exact-f32 MFMA and split-bf16 MFMA forms):
// the NT argument block, the dropout counter hash and the fused NT epilogue.
#pragma once
#include "common.hpp"

#include <utility>

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace gnnmp {

// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}


// Dropout keep decision for element `idx` of a call seeded with `seed`: murmur3's fmix32
// over (idx * golden + seed_lo) ^ seed_hi, top 24 bits compared with (1-p)·2^24.  32-bit
// arithmetic only (3 multiplies).  Mirrored bit for bit by oracle/dropout_hash.py.
constexpr uint32_t kDropGolden = 0x9E3779B1u;
// keep_elem from the premixed first term h0 = idx * kDropGolden + (uint32_t)seed, which a tile
// epilogue forms by additions (the map idx -> h0 is linear mod 2^32): two multiplies per element.
__device__ __forceinline__ bool keep_premixed(uint32_t h, uint64_t seed, uint32_t keep_thresh) {
  h ^= (uint32_t)(seed >> 32);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return (h >> 8) < keep_thresh;
}
__device__ __forceinline__ bool keep_elem(uint64_t seed, uint32_t idx, uint32_t keep_thresh) {
  uint32_t h = idx * kDropGolden + (uint32_t)seed;
  h ^= (uint32_t)(seed >> 32);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return (h >> 8) < keep_thresh;
}

constexpr int BN = 128;  // NT block columns (4 waves stacked by rows, each wave 4 x 32 columns)

struct NTArgs {
  int64_t M;
  int32_t Nc;
  const float* a1; int64_t lda1; int32_t k1;
  const float* a2; int64_t lda2; int32_t k2;
  const float* bt; int64_t ldb;
  const float* w1; const float* w2; int64_t ldw1, ldw2;  // alternative B: W1 [Nc, k1], W2 [Nc, k2]
  int32_t wvec2;                                          // W rows 8-byte aligned, k1/k2 even
  int32_t wvec;                                           // widest W row vector (1, 2, 4) for the nt2 staging
  float* c; int64_t ldc;
  const float* bias;
  int32_t relu;
  int32_t dropout; uint32_t keep_thresh; float drop_scale; uint64_t seed; const uint64_t* seed_ptr;
  const float* proj; int32_t nproj; float* z; int64_t ldz;
  int32_t a_bf16;  // A1/A2 hold bf16 (the float pointers are reinterpreted; ld in elements)
  int32_t c_bf16;  // C is stored as bf16 (RNE), and the projection reads the rounded values
  const float* mask; int64_t ldmask; float mask_scale;  // skinny kernels: C *= mask > 0 ? scale : 0
  // optional split image of [A1 | A2] (gnn_planes): 3 bf16 planes hi/mid/lo, plane p at
  // ap + p·ap_ps, row r at r·ap_ld; A1 in columns [0, k1), A2 in [ap_col2, ap_col2 + k2), zeros
  // elsewhere.  The weight-stationary kernel then stages A by plain copies (no split VALU).
  const uint16_t* ap; int32_t ap_ld; int32_t ap_col2; int64_t ap_ps;
  int32_t ap_h2;  // the image is a half-pair image (2 f16 planes hi / lo, gemm_ws.hip K7a-h)
  int32_t ap_exp; // half-pair: the image holds A · 2^ap_exp (undone in the epilogue's column scale)
  const uint32_t* kmask;  // optional dropout keep bits (half-pair NT): bit c of kmask[r·4 + c/32]
  float* colsum_part;     // optional (skinny-K NT): per-block column sums of the stored C, [nb][Nc]
  int32_t* rowexp;        // optional (in-kernel half-pair NT): per-row exponents E_r, max |A[r,:]| < 2^E_r
};

// the half-pair NT's B-image prep (ws_prep_h2_cols below)
struct H2Prep {
  const float* w1; const float* w2;  // w2 may be null (k2 = 0)
  int64_t ldw1, ldw2;
  int32_t k1, k2, Nc, col2;
  int32_t blocks;                    // k-steps of the image
  uint4* img; float* colscale;
  float a_unscale;                   // 2^-ap_exp of the A image (folded into colscale)
  int32_t gblocks;                   // 256-thread blocks of the column-form prep riding in K1 (0: none)
};

__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {  // RNE (v_cvt_pk_bf16_f32), NaN stays NaN
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

// Epilogue shared by the NT kernels: bias, ReLU, dropout, store, optional projection.
// acc[tm][t] is the 32x32 MFMA tile (rows wave·32·TM + tm·32 .., cols n0 + t·32 ..).
template <int TM, bool CBF = false>
__device__ __forceinline__ void nt_epilogue(const NTArgs& a, floatx16 (&acc)[TM][4], int64_t m0, int n0, int lane,
                                            int wave, uint64_t seed) {
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int64_t rbase = m0 + wave * 32 * TM + tm * 32 + 4 * (lane >> 5);
    const uint32_t hstep = (uint32_t)a.Nc * kDropGolden;  // premixed hash step per row
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int col = n0 + t * 32 + (lane & 31);
      const bool colok = col < a.Nc;
      const float bv = (a.bias && colok) ? a.bias[col] : 0.0f;
      const uint32_t h0 = ((uint32_t)rbase * (uint32_t)a.Nc + (uint32_t)col) * kDropGolden + (uint32_t)seed;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = rbase + (r & 3) + 8 * (r >> 2);
        float v = acc[tm][t][r] + bv;
        if (a.relu) v = fmaxf(v, 0.0f);
        if (a.dropout)  // == keep_elem(seed, row * Nc + col, thresh), bit for bit
          v = keep_premixed(h0 + (uint32_t)((r & 3) + 8 * (r >> 2)) * hstep, seed, a.keep_thresh) ? v * a.drop_scale
                                                                                                 : 0.0f;
        if (!colok) v = 0.0f;
        if constexpr (CBF) {
          const uint16_t b = f32_to_bf16(v);
          v = bf16_to_f32(b);
          if (a.c && row < a.M && colok) reinterpret_cast<uint16_t*>(a.c)[row * a.ldc + col] = b;
        } else {
          if (a.c && row < a.M && colok) a.c[row * a.ldc + col] = v;
        }
        acc[tm][t][r] = v;
      }
    }
    if (a.nproj > 0) {
      // z[row, q] = Σ_col h[row, col] · proj[q, col].  Each lane holds 4 columns of each of its
      // 16 rows; the 4 projection sums are reduced over the 32 lanes of a half-wave with a
      // reduce-and-split butterfly: xor 16 halves the q set, xor 8 halves it again, then
      // xor 4/2/1 finish one value — 6 shuffles per row instead of 4 x 5.
      float pw[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int col = n0 + t * 32 + (lane & 31);
          pw[q][t] = (q < a.nproj && col < a.Nc) ? a.proj[(int64_t)q * a.Nc + col] : 0.0f;
        }
      const bool hi16 = lane & 16, hi8 = lane & 8;
      const int qsel = (hi16 ? 2 : 0) + (hi8 ? 1 : 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float ps[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float sum = acc[tm][0][r] * pw[q][0];
          sum = fmaf(acc[tm][1][r], pw[q][1], sum);
          sum = fmaf(acc[tm][2][r], pw[q][2], sum);
          ps[q] = fmaf(acc[tm][3][r], pw[q][3], sum);
        }
        const float s0 = hi16 ? ps[0] : ps[2], s1 = hi16 ? ps[1] : ps[3];
        const float k0 = (hi16 ? ps[2] : ps[0]) + __shfl_xor(s0, 16);
        const float k1 = (hi16 ? ps[3] : ps[1]) + __shfl_xor(s1, 16);
        float m = (hi8 ? k1 : k0) + __shfl_xor(hi8 ? k0 : k1, 8);
        m += __shfl_xor(m, 4);
        m += __shfl_xor(m, 2);
        m += __shfl_xor(m, 1);
        const int64_t row = rbase + (r & 3) + 8 * (r >> 2);
        if ((lane & 7) == 0 && qsel < a.nproj && row < a.M) a.z[row * a.ldz + qsel] = m;
      }
    }
  }
}

constexpr int TN_THREADS = 1024;  // 16 waves: wave w owns dW rows (w&3)*32.. and k-tiles (w>>2)*3 .. +3
constexpr int KT_PER_WAVE = 3;
constexpr int KMAX = 4 * KT_PER_WAVE * 32;  // Kc <= 384
constexpr int TN_APITCH = KMAX;
constexpr int MAXPROJ = 4;

struct TNArgs {
  int64_t M;
  int32_t Nr;
  const float* g; int64_t ldg;
  const float* dz; int64_t lddz; const float* proj; int32_t nproj;
  const float* h; int64_t ldh; float hscale;
  float* gout; int64_t ldgout;
  const float* a1; int64_t lda1; int32_t k1;
  const float* a2; int64_t lda2; int32_t k2;
  float* slab; int64_t slab_stride;
  int64_t rows_per_block;
  int32_t want_db;
  int32_t a_bf16;  // A1/A2 hold bf16
  int32_t h_bf16;  // h holds bf16
  int32_t g_bf16;  // g (input) and gout (output) hold bf16 (the bf16-image TN)
  const uint16_t* ap; int32_t ap_ld; int32_t ap_col2; int64_t ap_ps;  // split image of [A1 | A2] (as NTArgs)
  int32_t ap_h2;  // half-pair image (2 f16 planes)
  int32_t ap_exp; // half-pair: the image holds A · 2^ap_exp (undone in the slab scale)
  const int32_t* rowexp;  // in-kernel half-pair TN: per-row exponents bounding A's rows (the NT's)
  const uint32_t* growmax;  // (ABI 25) the g form's max |G| per GNN_ROWMAX_ROWS rows (float bits), or null
  // (ABI 26) the half-pair dz form: dz[:, 0:ccols] formed in the TN as the CSC sum of u (null: read)
  const int32_t* cptr; const int32_t* cnbr; const float* cu; int64_t ldu; int32_t ccols;
};

// split-bf16 ("x3": each f32 operand = hi + mid + lo bf16, 6 MFMA products) launchers,
// defined in gemm_x3.hip.  Only the w1/w2 (in-place Linear weight) B form runs split.
void launch_nt_x3(const NTArgs& a, void* ws, size_t ws_bytes, hipStream_t st);
size_t nt_x3_workspace(int64_t k1, int64_t k2);
void launch_tn_x3(const TNArgs& a, int nblk, hipStream_t st);  // NPL = 3, or 1 when a_bf16
// the in-kernel half-pair forms (GNN_MATH_HALF_PAIR, gemm_x3.hip): f32 operands split into f16
// hi / lo with power-of-two scales (NT: per A row; TN: per row block), 3 products
bool nt_h2s_ok(const NTArgs& a);
size_t nt_h2s_workspace(int64_t k1, int64_t k2);
void launch_nt_h2s(const NTArgs& a, void* ws, hipStream_t st);
bool tn_h2s_ok(const TNArgs& a);
void launch_tn_h2s(const TNArgs& a, int nblk, hipStream_t st);

// weight-stationary persistent split-bf16 NT (gemm_ws.hip): B fragments resident in registers,
// one block per CU sweeping 32-row tiles.  nt_ws_ok: the shapes/epilogues it takes.  `img`: at
// least nt_x3_workspace(k1, k2) bytes of workspace for its pre-split B image (concatenated K).
bool nt_ws_ok(const NTArgs& a);
size_t nt_ws_tail_offset(int64_t k1, int64_t k2);
void launch_nt_ws(const NTArgs& a, uint4* img, hipStream_t st);
// the split-image forms (gemm_ws.hip NT, gemm_planes.hip TN): shapes they take, launchers
bool nt_planes_ok(const NTArgs& a);
// Image-A NT launch phases: the B-image prep, the GEMM, or both (gnn_gemm_nt_prep_b / b_ready)
constexpr int NT_PHASE_PREP = 1, NT_PHASE_RUN = 2, NT_PHASE_ALL = 3;
void launch_nt_ws_planes(const NTArgs& a, uint4* img, hipStream_t st, int phase = NT_PHASE_ALL);
// the bf16 image form (gemm_ws.hip): bf16 storage, one product per MFMA, LDS-DMA staged
bool nt_img16_ok(const NTArgs& a);
void launch_nt_img16(const NTArgs& a, uint4* img, hipStream_t st, int phase = NT_PHASE_ALL);
// the half-pair forms (f16 hi / lo images, 3 products): gemm_ws.hip / gemm_planes.hip
bool nt_h2_ok(const NTArgs& a);
H2Prep h2_prep_of(const NTArgs& a, uint4* img);  // the prep of the half-pair NT a over workspace img
// the half-pair NT's prep for a caller's NT params (gnn_sage_mean_fwd_h2's prep_b): GNN_OK and
// *out filled when p selects the half-pair NT with a large enough workspace, else UNSUPPORTED
gnn_status nt_h2_prep_from_params(const gnn_gemm_nt_params* p, H2Prep* out, const char* fn);
void launch_nt_h2(const NTArgs& a, uint4* img, hipStream_t st, int phase = NT_PHASE_ALL);
void launch_prep_h2(const H2Prep& p, hipStream_t st);  // ws_prep_h2_kernel over p (gemm_ws.hip)
bool tn_h2_ok(const TNArgs& a);
void launch_tn_h2(const TNArgs& a, int nblk, hipStream_t st, bool ks = false);
bool tn_planes_ok(const TNArgs& a);
void launch_tn_planes(const TNArgs& a, int nblk, hipStream_t st);
bool tn_img16_ok(const TNArgs& a);
void launch_tn_img16(const TNArgs& a, int nblk, hipStream_t st);
// 3 planes of one f32 split: hi = RNE(v), mid = RNE(v - hi), lo = RNE(v - hi - mid), exact sum
__device__ __forceinline__ void split3_pair(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  typedef __bf16 bf16x2_ __attribute__((ext_vector_type(2)));
  typedef float f32x2_ __attribute__((ext_vector_type(2)));
  h = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_{a, b}, bf16x2_));
  a -= __uint_as_float(h << 16);
  b -= __uint_as_float(h & 0xffff0000u);
  m = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_{a, b}, bf16x2_));
  a -= __uint_as_float(m << 16);
  b -= __uint_as_float(m & 0xffff0000u);
  l = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_{a, b}, bf16x2_));
}

// Half-pair split (gemm_ws.hip K7a-h): hi = RNE_f16(v), lo = RNE_f16((v - hi) · 2^11); the
// remainder is exact in f32 and v = hi + 2^-11 lo to 2^-22 |v| while hi and the scaled remainder
// are f16 normals (|v| >= 2^-13; below, an absolute 2^-36): the callers pre-scale A into
// [2^13, 2^14) (gnn_split_h2_f32 scale_exp) and G per block into [8, 16), and need |v| < 2^15.
__device__ __forceinline__ void split_h2_pair(float a, float b, uint32_t& h, uint32_t& l) {
  typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
  typedef float f32x2_ __attribute__((ext_vector_type(2)));
  const h2_ hv = __builtin_convertvector(f32x2_{a, b}, h2_);
  h = __builtin_bit_cast(uint32_t, hv);
  const float ra = (a - (float)hv[0]) * 2048.0f;
  const float rb = (b - (float)hv[1]) * 2048.0f;
  l = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_{ra, rb}, h2_));
}

// Two packed f16 values times a power of two (exact while the result stays in range).
__device__ __forceinline__ uint32_t h2_scale_pair(uint32_t h, float s) {
  typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
  typedef float f32x2_ __attribute__((ext_vector_type(2)));
  const h2_ v = __builtin_bit_cast(h2_, h);
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_{(float)v[0] * s, (float)v[1] * s}, h2_));
}

// VALU kernels for the narrow output-layer shapes (gemm_skinny.hip).  launch_nt_skinny returns
// false (launching nothing) when the shape/epilogue is outside its envelope.
bool launch_nt_skinny(const NTArgs& a, hipStream_t st);
int nt_skinny_k_blocks(const NTArgs& a);  // grid of the skinny-K form (its colsum_part rows); 0: not that form
int tn_skinny_blocks(int64_t M);
bool tn_skinny_ok(const TNArgs& a);
void launch_tn_skinny(const TNArgs& a, int nblk, hipStream_t st);


// ---- the half-pair NT's B image (K7a-h).  Per k-step s, plane p (hi' = 2^11 hi, hi, lo), slot
// 2n + khalf: the 8 halves of column n, k = 16s + 8·khalf .. +8, of w_n · 2^-e_n, where 2^-e_n
// brings the column's largest |w| into [8, 16) (a power of two: exact); colscale[n] =
// 2^(e_n - 11 - ap_exp), which also undoes the A image's pre-scale.
// Column form (round 6): ONE WAVE PER OUTPUT COLUMN n — B's column n is row n of the Linear
// weights, contiguous — so a wave loads its whole column (12 loads per lane, all issued before the
// first use, indices clamped, the excess masked to 0), takes the max with a butterfly, stages the
// column's image row in LDS and writes its 2·NKS (k-step, khalf) slots of all three planes.  One
// load round trip per wave instead of the k-step form's all-columns sweep per block (32 / CPP
// dependent rounds per wave: the riding prep was K1's critical path on a strong-scaling shard,
// 22.0 vs 17.9 us gather alone at 8 shards).  The grid covers all BN columns (zeros past Nc);
// the image is bit-identical to the k-step form's (the same per-element arithmetic; a max is
// order-free).  Needs k1, k2 <= 384 and 16·NKS <= 384 (nt_h2_ok: <= 336).
__device__ __forceinline__ float h2_col_exp2(float m) {  // 2^e with m · 2^-e in [8, 16); 1 for m = 0
  if (!(m > 0.f) || !isfinite(m)) return 1.0f;
  int E;
  frexpf(m, &E);  // m in [2^(E-1), 2^E)
  return ldexpf(1.0f, E - 4);
}
template <int NTH>
__device__ __forceinline__ void ws_prep_h2_cols(const H2Prep& a, int blk) {
  constexpr int NW = NTH / 64;
  constexpr int ROW = 16 * 24 + 4;                 // an image row (<= 384 columns) per wave
  __shared__ float wrow[NW][ROW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = blk * NW + wave;                   // this wave's column
  if (n >= BN) return;                             // (wave-uniform; no block barrier below)
  const bool live = n < a.Nc;
  const int nc = live ? n : 0;
  const int k1m = a.k1 - 1, k2m = a.k2 > 0 ? a.k2 - 1 : 0;
  const float* w1 = a.w1 + (int64_t)nc * a.ldw1;
  const float* w2 = (a.w2 ? a.w2 : a.w1) + (int64_t)nc * (a.w2 ? a.ldw2 : a.ldw1);
  float v[12];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    v[i] = w1[min(lane + 64 * i, k1m)];
    v[6 + i] = w2[min(lane + 64 * i, k2m)];
  }
  float* row = wrow[wave];
  const int ncols = 16 * a.blocks;
  for (int kk = lane; kk < ncols; kk += 64) row[kk] = 0.f;
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    m = fmaxf(m, lane + 64 * i < a.k1 ? fabsf(v[i]) : 0.f);
    m = fmaxf(m, lane + 64 * i < a.k2 ? fabsf(v[6 + i]) : 0.f);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  const float sc = live ? h2_col_exp2(m) : 1.0f;
  if (lane == 0) a.colscale[n] = sc * (1.0f / 2048.0f) * a.a_unscale;  // powers of two: exact
  // (the zeroing stores above precede these in this wave's LDS order)
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int k = lane + 64 * i;
    if (live && k < a.k1) row[k] = v[i];
    if (live && k < a.k2) row[a.col2 + k] = v[6 + i];
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's row is in LDS
  __builtin_amdgcn_wave_barrier();
  const float inv = 1.0f / sc;  // a power of two: exact
  for (int q = lane; q < 2 * a.blocks; q += 64) {
    const int s = q >> 1, kh = q & 1;
    uint32_t hw[4], lw[4], pw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v0 = row[16 * s + 8 * kh + 2 * j] * inv, v1 = row[16 * s + 8 * kh + 2 * j + 1] * inv;
      split_h2_pair(v0, v1, hw[j], lw[j]);
      pw[j] = h2_scale_pair(hw[j], 2048.0f);
    }
    const int64_t slot = 2 * n + kh;
    a.img[((int64_t)s * 3 + 0) * 256 + slot] = make_uint4(pw[0], pw[1], pw[2], pw[3]);
    a.img[((int64_t)s * 3 + 1) * 256 + slot] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    a.img[((int64_t)s * 3 + 2) * 256 + slot] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
  }
}
constexpr int WS_PREP_THREADS = 1024;

}  // namespace gnnmp
