// K7x — fp32 GEMMs of K7 on the bf16 matrix cores by operand splitting ("x3").
//
// gfx950 runs v_mfma_f32_32x32x16_bf16 at 16x the FLOP rate of the exact-f32
// v_mfma_f32_32x32x2_f32 (MI355X_MICROARCH.md, Matrix cores).  Each f32 operand is split on the
// fly into three bf16 terms, a = hi + mid + lo, by round-to-nearest conversions whose remainders
// are exact in f32 (hi keeps 8 significant bits, mid the next 8, lo the rest: the sum is exact
// for every normal f32).  The product keeps the six terms of magnitude >= 2^-16 relative,
//     a·b ≈ hh + hm + mh + hl + lh + mm     (dropped: ml + lm + ll <= ~2^-23 |a·b|, unbiased)
// accumulated in f32 by the MFMA, i.e. fp32-accurate results at 16/6 = 2.7x the exact-f32 MFMA
// peak.  The splits happen while staging into LDS (VALU, hidden under the MFMAs); both operands
// are K-contiguous bf16 planes read as ds_read_b128 fragments (pitch ≡ 12 or 20 dwords mod 64:
// conflict-free b128 lane groups).
//
// NT (forward, replaces lin_l/lin_r + ReLU + dropout, gnn.py:41-44,49-51):
//   C = epi([A1 | A2] · [W1 | W2]ᵀ), W read in place from the Linear weights; epilogue shared
//   with the f32 kernels (gemm_common.hpp: bias, ReLU, counter-hash dropout, projection).
// TN (backward weight gradients): dW = Gᵀ·[A1 | A2] over row chunks of 16 (one MFMA k-step),
//   G formed on the fly from dz·P (or g) and the ReLU/dropout mask of h; per-block slabs reduced
//   in a fixed order by gemm_f32.hip's slab_reduce_kernel.  Atomic-free and deterministic.
#include "gemm_common.hpp"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

namespace gnnmp {
namespace {

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {  // RNE, a in the low half
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v{a, b}, bf16x2v));
}

// (a, b) -> three packed bf16 pairs w[0] (hi), w[1] (mid), w[2] (lo); a = hi + mid + lo exactly.
__device__ __forceinline__ void split_pair(float a, float b, uint32_t (&w)[3]) {
  w[0] = pk_bf16(a, b);
  a -= __uint_as_float(w[0] << 16);
  b -= __uint_as_float(w[0] & 0xffff0000u);
  w[1] = pk_bf16(a, b);
  a -= __uint_as_float(w[1] << 16);
  b -= __uint_as_float(w[1] & 0xffff0000u);
  w[2] = pk_bf16(a, b);
}

__device__ __forceinline__ floatx16 mfma6(const bf16x8 (&x)[3], const bf16x8 (&y)[3], floatx16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[1], y[1], c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[2], y[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[1], y[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[0], c, 0, 0, 0);
  return c;
}

template <int NPL>
__device__ __forceinline__ floatx16 mfma_planes(const bf16x8 (&x)[NPL], const bf16x8 (&y)[NPL], floatx16 c) {
  if constexpr (NPL == 3) return mfma6(x, y, c);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[0], c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 lds_frag(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// ---- the in-kernel half-pair form (GNN_MATH_HALF_PAIR, round 6).  An f32 operand v, scaled by a
// power of two s into |v·s| < 2^14 (A) or < 16 (G), is held as two f16 planes hi = RNE_f16(v·s),
// lo = RNE_f16((v·s − hi)·2^11) (gemm_common.hpp split_h2_pair); the other operand carries three
// (hi' = 2^11 hi, hi, lo), and a product is three f16 MFMAs, lo·hi + hi·lo + hi·hi' (the dropped
// lo·lo is 2^-22 relative) — the arithmetic of the half-pair image kernels with the split done while
// staging, so it serves operands that change every step (SAGE-ResBN's hidden layers).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f16x8 lds_frag16(const uint16_t* p) { return *reinterpret_cast<const f16x8*>(p); }
__device__ __forceinline__ floatx16 mfma_h2(const f16x8& x_hi, const f16x8& x_lo, const f16x8& y_hi2,
                                            const f16x8& y_hi, const f16x8& y_lo, floatx16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(x_lo, y_hi, c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(x_hi, y_lo, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(x_hi, y_hi2, c, 0, 0, 0);
  return c;
}
// 2^(14 − E) for a row bound m < 2^E (A rows into |v·s| < 2^14); E = 0 for m = 0, 128 non-finite
__device__ __forceinline__ int h2_row_exp(float m) {
  if (!isfinite(m)) return 128;
  int E = 0;
  if (m > 0.f) frexpf(m, &E);
  return E;
}

// p + e elements of a buffer that holds f32 or (BF) bf16
template <bool BF>
__device__ __forceinline__ const float* elem_ptr(const float* p, int64_t e) {
  if constexpr (BF) return reinterpret_cast<const float*>(reinterpret_cast<const uint16_t*>(p) + e);
  else return p + e;
}

// ------------------------------------------------------------------------------------- NT
// Stage rows [r0, r0+ROWS) x [k0, k0+KC) of a K-contiguous f32 operand into registers, in units
// of U consecutive k per thread, each loaded as U/V vectors of V floats (V | k1, k2, ld).
// Addresses are clamped (never data-dependent), so the prefetch stays in flight across the
// MFMAs; masking happens at the split/store.
template <int V, int U, int KC, int ROWS, bool BF = false>
__device__ __forceinline__ void x3_load_rows(const float* X, int64_t ldx, int64_t r0, int64_t rows, int k0,
                                             int klen, float* reg) {
  if constexpr (BF) {  // bf16 rows (ld in elements): V bf16 per load, widened to f32 (exact)
    const uint16_t* X16 = reinterpret_cast<const uint16_t*>(X);
    constexpr int UPR = KC / U;
#pragma unroll
    for (int i = 0; i < ROWS * KC / 256 / U; ++i) {
      const int v = threadIdx.x + 256 * i;
      const int r = v / UPR;
      const int k = (v % UPR) * U;
      int64_t row = r0 + r;
      row = row < rows ? row : rows - 1;
      const uint16_t* p = X16 + row * ldx + k0;
#pragma unroll
      for (int j = 0; j < U; j += V) {
        const int kk = k + j < klen ? k + j : 0;
        if constexpr (V == 4) {
          const uint2 t = *reinterpret_cast<const uint2*>(p + kk);
          reg[i * U + j] = __uint_as_float(t.x << 16); reg[i * U + j + 1] = __uint_as_float(t.x & 0xffff0000u);
          reg[i * U + j + 2] = __uint_as_float(t.y << 16); reg[i * U + j + 3] = __uint_as_float(t.y & 0xffff0000u);
        } else if constexpr (V == 2) {
          const uint32_t t = *reinterpret_cast<const uint32_t*>(p + kk);
          reg[i * U + j] = __uint_as_float(t << 16); reg[i * U + j + 1] = __uint_as_float(t & 0xffff0000u);
        } else {
          reg[i * U + j] = bf16_to_f32(p[kk]);
        }
      }
    }
    return;
  }
  constexpr int UPR = KC / U;
#pragma unroll
  for (int i = 0; i < ROWS * KC / 256 / U; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int r = v / UPR;
    const int k = (v % UPR) * U;
    int64_t row = r0 + r;
    row = row < rows ? row : rows - 1;
    const float* p = X + row * ldx + k0;
#pragma unroll
    for (int j = 0; j < U; j += V) {
      const int kk = k + j < klen ? k + j : 0;
      if constexpr (V == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p + kk);
        reg[i * U + j] = t.x; reg[i * U + j + 1] = t.y; reg[i * U + j + 2] = t.z; reg[i * U + j + 3] = t.w;
      } else if constexpr (V == 2) {
        const float2 t = *reinterpret_cast<const float2*>(p + kk);
        reg[i * U + j] = t.x; reg[i * U + j + 1] = t.y;
      } else {
        reg[i * U + j] = p[kk];
      }
    }
  }
}

// Split and store into three bf16 planes L[p * ROWS * PITCH + r * PITCH + k] (one b32 / b64 /
// b128 store per plane for U = 2 / 4 / 8); zero outside (rows, klen).
template <int U, int KC, int ROWS, int PITCH, int NPL = 3>
__device__ __forceinline__ void x3_store_rows(uint16_t* L, int64_t r0, int64_t rows, int klen, const float* reg) {
  constexpr int UPR = KC / U;
  constexpr int PL = ROWS * PITCH;
#pragma unroll
  for (int i = 0; i < ROWS * KC / 256 / U; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int r = v / UPR;
    const int k = (v % UPR) * U;
    const bool rok = r0 + r < rows;
    uint32_t w[U / 2][3];
#pragma unroll
    for (int j = 0; j < U / 2; ++j) {
      const int kk = k + 2 * j;
      const float e0 = (rok && kk < klen) ? reg[i * U + 2 * j] : 0.0f;
      const float e1 = (rok && kk + 1 < klen) ? reg[i * U + 2 * j + 1] : 0.0f;
      split_pair(e0, e1, w[j]);
    }
    uint16_t* d = L + r * PITCH + k;
#pragma unroll
    for (int p = 0; p < NPL; ++p) {
      if constexpr (U == 8) *reinterpret_cast<uint4*>(d + p * PL) = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
      else if constexpr (U == 4) *reinterpret_cast<uint2*>(d + p * PL) = make_uint2(w[0][p], w[1][p]);
      else *reinterpret_cast<uint32_t*>(d + p * PL) = w[0][p];
    }
  }
}

// The half-pair form of x3_store_rows: unit i's row scaled by sc[i] (a power of two, exact), two
// f16 planes hi / lo; zero outside (rows, klen).
template <int U, int KC, int ROWS, int PITCH>
__device__ __forceinline__ void h2_store_rows(uint16_t* L, int64_t r0, int64_t rows, int klen, const float* reg,
                                              const float* sc) {
  constexpr int UPR = KC / U;
  constexpr int PL = ROWS * PITCH;
#pragma unroll
  for (int i = 0; i < ROWS * KC / 256 / U; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int r = v / UPR;
    const int k = (v % UPR) * U;
    const bool rok = r0 + r < rows;
    uint32_t w[U / 2][2];
#pragma unroll
    for (int j = 0; j < U / 2; ++j) {
      const int kk = k + 2 * j;
      const float e0 = (rok && kk < klen) ? reg[i * U + 2 * j] * sc[i] : 0.0f;
      const float e1 = (rok && kk + 1 < klen) ? reg[i * U + 2 * j + 1] * sc[i] : 0.0f;
      split_h2_pair(e0, e1, w[j][0], w[j][1]);
    }
    uint16_t* d = L + r * PITCH + k;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if constexpr (U == 8) *reinterpret_cast<uint4*>(d + p * PL) = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
      else if constexpr (U == 4) *reinterpret_cast<uint2*>(d + p * PL) = make_uint2(w[0][p], w[1][p]);
      else *reinterpret_cast<uint32_t*>(d + p * PL) = w[0][p];
    }
  }
}

// B pre-split once per call (BV == 0 kernels): per KC=16 chunk c, image [plane][n 128][16 k]
// bf16 (12 KB, zero outside k < klen, n < Nc), copied to LDS as 3 b128 per thread per chunk.
__global__ __launch_bounds__(256) void x3_presplit_b_kernel(NTArgs a, uint4* __restrict__ img, int nch1,
                                                            int nchunks, int swz = 0) {
  const int idx = blockIdx.x * 256 + threadIdx.x;  // (chunk, n, khalf)
  if (blockIdx.x == 0 && threadIdx.x < 4) img[(int64_t)nchunks * 3 * 256 + threadIdx.x] = make_uint4(0, 0, 0, 0);
  if (idx >= nchunks * 256) return;
  const int c = idx >> 8, n = (idx & 255) >> 1, kh = idx & 1;
  const float* W; int64_t ldw; int k0, klen;
  if (c < nch1) { W = a.w1; ldw = a.ldw1; k0 = c * 16; klen = min(16, a.k1 - k0); }
  else { W = a.w2; ldw = a.ldw2; k0 = (c - nch1) * 16; klen = min(16, a.k2 - k0); }
  float e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kh + j;
    e[j] = (n < a.Nc && k < klen) ? W[(int64_t)n * ldw + k0 + k] : 0.0f;
  }
  uint32_t w[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j) split_pair(e[2 * j], e[2 * j + 1], w[j]);
  // swz (the LDS-DMA kernel's image): the k-half of row n is stored at kh ^ bit 3 of n, so the
  // lane-linear DMA copy lands conflict-free for the ds_read_b128 fragment reads
  const int slot = swz ? 2 * n + (kh ^ ((n >> 3) & 1)) : (idx & 255);
#pragma unroll
  for (int p = 0; p < 3; ++p) img[((int64_t)c * 3 + p) * 256 + slot] = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
}

template <int KC>
__device__ __forceinline__ void x3_chunk(const NTArgs& a, int c, int nch1, const float*& A, int64_t& lda,
                                         const float*& W, int64_t& ldw, int& k0, int& klen) {
  if (c < nch1) { A = a.a1; lda = a.lda1; W = a.w1; ldw = a.ldw1; k0 = c * KC; klen = min(KC, a.k1 - k0); }
  else { A = a.a2; lda = a.lda2; W = a.w2; ldw = a.ldw2; k0 = (c - nch1) * KC; klen = min(KC, a.k2 - k0); }
}

// Block: 4 waves, wave w owns rows w·32·TM .. (+32·TM) x all 128 columns (the epilogue's
// projection needs whole rows in one wave).  K in chunks of KC through double-buffered LDS,
// fed by a ring of D register stages: chunk c's loads are issued D chunks ahead, so D chunks
// of A (BM x KC f32) are in flight per block while the MFMAs run (the split MFMA work per chunk
// is short; without depth the loop waits on HBM latency).  One barrier per chunk.
// NPL = 3: f32 operands split (6 products); NPL = 1 with ABF: bf16 operands as stored, B rounded
// to bf16 (the image's hi plane), one product (the bf16-storage path); CBF: C stored as bf16.
constexpr int NT_PIPE = 32, NT_HINTS = 64;  // gemm_nt_x3_kernel schedule flags (the bf16-storage form)

template <int KC, int TM, int AV, int AU, int BV, int D, int NPL = 3, bool ABF = false, bool CBF = false, int SCHED = 0>
__global__ __launch_bounds__(256) void gemm_nt_x3_kernel(NTArgs a, const uint4* __restrict__ bimg) {
  constexpr int P = KC + 8;  // bf16 per LDS row: 24 or 40 (12 / 20 dwords)
  constexpr int BM = 128 * TM;
  constexpr int APL = BM * P, BPL = BN * P;
  constexpr int AREG = BM * KC / 256, BREG = BN * KC / 256;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][NPL * APL];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][NPL * BPL];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int nch1 = (a.k1 + KC - 1) / KC;
  const int nchunks = nch1 + (a.k2 + KC - 1) / KC;
  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;

  floatx16 acc[TM][4];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][t][r] = 0.0f;

  // BV > 0: B split on the fly from the f32 weights; BV == 0: B copied from the pre-split image
  constexpr int BU = BV < 2 ? 2 : BV;
  constexpr int RB = BV == 0 ? 12 : BREG;  // image: 3 planes x uint4 per thread (KC = 16)
  static_assert(BV > 0 || KC == 16, "pre-split B image is cut in 16-deep chunks");
  float ra[D][AREG], rb[D][RB];
  auto load = [&](int c, float* rA, float* rB) {
    const float *A, *W; int64_t lda, ldw; int k0, klen;
    x3_chunk<KC>(a, c, nch1, A, lda, W, ldw, k0, klen);
    x3_load_rows<AV, AU, KC, BM, ABF>(A, lda, m0, a.M, k0, klen, rA);
    if constexpr (BV == 0) {
#pragma unroll
      for (int p = 0; p < NPL; ++p) {
        const uint4 t = bimg[((int64_t)c * 3 + p) * 256 + threadIdx.x];
        rB[4 * p] = __uint_as_float(t.x); rB[4 * p + 1] = __uint_as_float(t.y);
        rB[4 * p + 2] = __uint_as_float(t.z); rB[4 * p + 3] = __uint_as_float(t.w);
      }
    } else {
      x3_load_rows<BV, BU, KC, BN>(W, ldw, n0, a.Nc, k0, klen, rB);
    }
  };
  auto store = [&](int c, int buf, const float* rA, const float* rB) {
    const float *A, *W; int64_t lda, ldw; int k0, klen;
    x3_chunk<KC>(a, c, nch1, A, lda, W, ldw, k0, klen);
    x3_store_rows<AU, KC, BM, P, NPL>(As[buf], m0, a.M, klen, rA);
    if constexpr (BV == 0) {
      const int n = threadIdx.x >> 1, kh = threadIdx.x & 1;
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        *reinterpret_cast<uint4*>(&Bs[buf][p * BPL + n * P + 8 * kh]) =
            make_uint4(__float_as_uint(rB[4 * p]), __float_as_uint(rB[4 * p + 1]), __float_as_uint(rB[4 * p + 2]),
                       __float_as_uint(rB[4 * p + 3]));
    } else {
      x3_store_rows<BU, KC, BN, P, NPL>(Bs[buf], n0, a.Nc, klen, rB);
    }
  };
  const int fr = (lane & 31) * P + 8 * (lane >> 5);
  auto compute = [&](int buf, int c) {
    const int klen = c < nch1 ? min(KC, a.k1 - c * KC) : min(KC, a.k2 - (c - nch1) * KC);
    const uint16_t* Ab = As[buf] + wave * 32 * TM * P + fr;
    const uint16_t* Bb = Bs[buf] + fr;
#pragma unroll
    for (int s = 0; s < KC / 16; ++s) {
      if (KC == 16 || 16 * s < klen) {  // KC == 16: every chunk has klen >= 1 (no branch)
        bf16x8 af[TM][NPL], bf[4][NPL];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int p = 0; p < NPL; ++p) af[tm][p] = lds_frag(Ab + p * APL + tm * 32 * P + 16 * s);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int p = 0; p < NPL; ++p) bf[t][p] = lds_frag(Bb + p * BPL + t * 32 * P + 16 * s);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int tm = 0; tm < TM; ++tm) acc[tm][t] = mfma_planes<NPL>(af[tm], bf[t], acc[tm][t]);
      }
    }
  };

  // Loads are unconditional (a clamped chunk index: the tail re-reads the last chunk) so the
  // main loop is straight-line code and the compiler's vmcnt waits leave the other D-1 stages
  // in flight; a branch around a load makes it drain every stage at the next store.
#pragma unroll
  for (int d = 0; d < D; ++d) load(min(d, nchunks - 1), ra[d], rb[d]);
  if constexpr ((SCHED & NT_PIPE) != 0) {
    // software-pipelined order: between two barriers, stage chunk c+1 into the other buffer
    // while the MFMAs of chunk c run, so VALU splits / LDS writes interleave with the MFMAs
    store(0, 0, ra[0], rb[0]);
    load(min(D, nchunks - 1), ra[0], rb[0]);
    int c = 0;
    for (; c + D < nchunks; c += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int cc = c + d;  // cc + 1 < nchunks for all d here
        const int d1 = (d + 1) % D;
        __syncthreads();
        store(cc + 1, (cc + 1) & 1, ra[d1], rb[d1]);
        load(min(cc + 1 + D, nchunks - 1), ra[d1], rb[d1]);
        compute(cc & 1, cc);
        if constexpr ((SCHED & NT_HINTS) != 0) {  // interleave: per MFMA, a few VALU / DS ops
#pragma unroll
          for (int i = 0; i < 4 * TM * (NPL == 3 ? 6 : 1) * (KC / 16); ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
          }
        }
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int cc = c + d;
      if (cc < nchunks) {
        const int d1 = (d + 1) % D;
        __syncthreads();
        if (cc + 1 < nchunks) store(cc + 1, (cc + 1) & 1, ra[d1], rb[d1]);
        compute(cc & 1, cc);
      }
    }
    nt_epilogue<TM, CBF>(a, acc, m0, n0, lane, wave, seed);
    return;
  }
  int c0 = 0;
  for (; c0 + D <= nchunks; c0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int c = c0 + d;
      const int buf = c & 1;
      store(c, buf, ra[d], rb[d]);  // buf last read by compute(c - 2): behind barrier c - 1
      __syncthreads();
      load(min(c + D, nchunks - 1), ra[d], rb[d]);
      compute(buf, c);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) {  // tail: the last nchunks mod D chunks, already loaded
    const int c = c0 + d;
    if (c < nchunks) {
      store(c, c & 1, ra[d], rb[d]);
      __syncthreads();
      compute(c & 1, c);
    }
  }
  nt_epilogue<TM, CBF>(a, acc, m0, n0, lane, wave, seed);
}

template <int KC, int TM, int AV, int AU, int D>
void launch_nt_x3_b(const NTArgs& a, const uint4* bimg, hipStream_t st) {
  dim3 grid((unsigned)ceil_div(a.M, 128 * TM), (unsigned)ceil_div(a.Nc, BN));
  if (bimg) gemm_nt_x3_kernel<KC, TM, AV, AU, 0, D><<<grid, 256, 0, st>>>(a, bimg);
  else if (a.wvec == 4) gemm_nt_x3_kernel<KC, TM, AV, AU, 4, D><<<grid, 256, 0, st>>>(a, nullptr);
  else if (a.wvec == 2) gemm_nt_x3_kernel<KC, TM, AV, AU, 2, D><<<grid, 256, 0, st>>>(a, nullptr);
  else gemm_nt_x3_kernel<KC, TM, AV, AU, 1, D><<<grid, 256, 0, st>>>(a, nullptr);
}

template <int KC, int TM, int D, int AU>
void launch_nt_x3_a(const NTArgs& a, int av, const uint4* bimg, hipStream_t st) {
  if (av == 4) launch_nt_x3_b<KC, TM, 4, (AU < 4 ? 4 : AU), D>(a, bimg, st);
  else if (av == 2) launch_nt_x3_b<KC, TM, 2, AU, D>(a, bimg, st);
  else launch_nt_x3_b<KC, TM, 1, AU, D>(a, bimg, st);
}

// ---- the in-kernel half-pair NT (GNN_MATH_HALF_PAIR, round 6): C = epi([A1 | A2] · [W1 | W2]ᵀ) for
// f32 A changing every step (SAGE-ResBN's hidden layers: K = 128, N = 64 forward, K = 64, N = 128
// for the input gradient).  Block: 128 rows x NTL·32 columns, 4 waves of 32 rows.  ALL NCH 16-deep
// chunks of the block's A rows are loaded up front (8 floats per thread per chunk, every load in
// flight at once: the chunk loop then waits only on LDS), which also gives each row its exponent
// E_r (max_k |A[r,k]| < 2^E_r, a butterfly over the row's 4 lanes); A is staged per chunk as f16
// hi / lo of A[r,:]·2^(14 − E_r) and B from the half-pair image (ws_prep_h2_cols, k-step s = chunk
// s) two chunks ahead; three f16 products per k-step; the epilogue multiplies row r, column n by
// 2^(E_r − 14)·2^(e_n − 11) (exact) before the shared bias / ReLU / dropout / projection epilogue.
// NTL = 2 (N <= 64): the B columns past 64 are neither staged nor multiplied.
template <int NCH, int NTL, int AV>
__global__ __launch_bounds__(256) void gemm_nt_h2s_kernel(NTArgs a, const uint4* __restrict__ bimg) {
  constexpr int KC = 16, P = KC + 8, BM = 128, AU = 4, UPR = KC / AU;
  constexpr int NBC = NTL * 32;                    // B columns staged
  constexpr int APL = BM * P, BPL = NBC * P;
  constexpr int AREG = BM * KC / 256, NUA = AREG / AU;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][2 * APL];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][3 * BPL];
  __shared__ float rsc[BM];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int nch1 = a.k1 / KC;
  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;
  float ra[NCH][AREG];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const float* A = c < nch1 ? a.a1 : a.a2;
    const int64_t lda = c < nch1 ? a.lda1 : a.lda2;
    const int k0 = (c < nch1 ? c : c - nch1) * KC;
    x3_load_rows<AV, AU, KC, BM>(A, lda, m0, a.M, k0, KC, ra[c]);
  }
  const bool bon = threadIdx.x < 2 * NBC;          // slot 2n + khalf of a staged column
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));  // (a plain vector: stays in registers)
  u32x4v rb[2][3];
  const u32x4v* bim = reinterpret_cast<const u32x4v*>(bimg);
  auto load_b = [&](int s, int c) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 3; ++p) rb[s][p] = bim[((int64_t)c * 3 + p) * 256 + threadIdx.x];
  };
  load_b(0, 0);
  load_b(1, min(1, NCH - 1));
  // the row exponents (rows fixed across chunks: unit i holds row (tid + 256 i) / UPR)
  float asc[NUA];
  {
    float mx[NUA];
#pragma unroll
    for (int i = 0; i < NUA; ++i) {
      mx[i] = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int j = 0; j < AU; ++j) mx[i] = fmaxf(mx[i], fabsf(ra[c][i * AU + j]));
#pragma unroll
      for (int o = 1; o < UPR; o <<= 1) mx[i] = fmaxf(mx[i], __shfl_xor(mx[i], o));
      const int r = (threadIdx.x + 256 * i) / UPR;
      const int E = h2_row_exp(mx[i]);
      asc[i] = E == 128 ? 1.0f : ldexpf(1.0f, 14 - E);
      if ((threadIdx.x % UPR) == 0) {
        rsc[r] = E == 128 ? 1.0f : ldexpf(1.0f, E - 14);
        if (a.rowexp && m0 + r < a.M) a.rowexp[m0 + r] = E;
      }
    }
  }
  floatx16 acc[1][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][t][r] = 0.0f;
  const int fr = (lane & 31) * P + 8 * (lane >> 5);
  const int bn = threadIdx.x >> 1, bkh = threadIdx.x & 1;
  static_for<NCH>([&](auto cc) __attribute__((always_inline)) {  // (static: ra / rb stay in registers)
    constexpr int c = decltype(cc)::value;
    constexpr int buf = c & 1;
    h2_store_rows<AU, KC, BM, P>(As[buf], m0, a.M, KC, ra[c], asc);
    if (bon) {
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x4v*>(&Bs[buf][p * BPL + bn * P + 8 * bkh]) = rb[buf][p];
    }
    __syncthreads();
    if constexpr (c + 2 < NCH) load_b(buf, c + 2);
    f16x8 af[2], bf[NTL][3];
    const uint16_t* Ab = As[buf] + wave * 32 * P + fr;
#pragma unroll
    for (int p = 0; p < 2; ++p) af[p] = lds_frag16(Ab + p * APL);
#pragma unroll
    for (int t = 0; t < NTL; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p) bf[t][p] = lds_frag16(Bs[buf] + fr + p * BPL + t * 32 * P);
#pragma unroll
    for (int t = 0; t < NTL; ++t) acc[0][t] = mfma_h2(af[0], af[1], bf[t][0], bf[t][1], bf[t][2], acc[0][t]);
  });
  const float* csc = reinterpret_cast<const float*>(bimg + (int64_t)NCH * 3 * 256);
#pragma unroll
  for (int t = 0; t < NTL; ++t) {  // undo the row and column scales (powers of two: exact)
    const float cs = csc[t * 32 + (lane & 31)];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][t][r] *= rsc[wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)] * cs;
  }
  nt_epilogue<1, false>(a, acc, m0, 0, lane, wave, seed);
}

// ------------------------------------------------------------------------------------- TN
constexpr int TMC = 16;            // rows per chunk = one MFMA k-step
constexpr int TP = TMC + 8;        // bf16 per transposed LDS row (12 dwords: conflict-free b128)
constexpr int TGPL = 128 * TP;     // G plane: [n][m]
constexpr int TAPL = KMAX * TP;    // A plane: [k][m]
constexpr int TX_THREADS = 256;    // 4 waves, one per SIMD (512 registers each)
constexpr int TX_AS = 3;           // A unit slots per thread (u = tid + 256·s < 768)

// Staging: every thread owns TX_AS A slots and one G slot (plus a g slot for the g form with
// MASK), each 8 consecutive rows of one column described by (base, ld, octet) and loaded by
// the SAME straight-line code whatever the role, so the ring of D register stages keeps D-1
// chunks of loads in flight across the store/barrier (a branch around a load would make the
// compiler drain every stage).
//   A slot s: u = tid + 256·s -> column k = u mod KP, rows 8·(u / KP) ..  if u < 2·KP, else idle
//   G slot:   column n = tid mod 128, rows 8·(tid / 128) ..: h[:, n] (MASK) or g[:, n]
// Idle slots load a fixed valid address.  dz (PROJ) is staged one chunk ahead into a 2-slot
// LDS ring (16 rows x 4) by threads 0..63, so G(c) = (dz·P) ⊙ mask is formed at store(c)
// from LDS instead of 32 registers of replicated dz rows per thread.
// NPL = 3: f32 operands split (6 products).  NPL = 1: the bf16-storage path — A (ABF) and h
// (HBF) are read as bf16, G is rounded to bf16, one product per MFMA.
// HALFN (Nr <= 64): waves 0-1 / 2-3 take the two 32-row halves of the output for the first /
// second half of the k-tiles (KT per wave), instead of waves 2-3 running MFMAs on all-zero rows.
// H2S (round 6, GNN_MATH_HALF_PAIR; the plain g form): the in-kernel half-pair form.  Before the
// chunk loop (behind chunk 0's loads) the block takes E_A = max row_exp[r] over its rows (the
// forward NT's row bounds of the same A) and E_G from max |g| over its rows (one pass, float4
// pieces), stages A as f16 hi / lo of A·2^(14 − E_A) and G as hi' / hi / lo of G·2^(4 − E_G), runs
// three products per k-tile, and writes acc·2^(E_A − 14)·2^(E_G − 15) to its slab (exact).
template <bool PROJ, bool MASK, int D, int KT, int NPL = 3, bool ABF = false, bool HBF = false, int PIPE = 0,
          bool GOUT = true, bool HALFN = false, bool H2S = false>
__device__ __forceinline__ void gemm_tn_split_body(const TNArgs& a) {
  static_assert(!H2S || (!PROJ && !MASK && !GOUT && NPL == 3 && !ABF && PIPE == 0), "half-pair: plain g form, f32");
  constexpr int NS = TX_AS + ((!PROJ && MASK) ? 2 : 1);  // + G slot (+ g slot)
  constexpr int GS = TX_AS;                              // the G slot index
  constexpr int APN = H2S ? 2 : NPL;                     // A planes (H2S: hi, lo; G keeps 3: hi', hi, lo)
  // A columns staged: the k-tiles the waves multiply (round 6: sized by KT, not KMAX — the narrow
  // shapes then fit two blocks per CU, and a latency-bound chunk loop gets twice the loads in flight)
  constexpr int KPM = (HALFN ? 2 * KT : KT) * 32;
  constexpr int TAPLK = KPM * TP;
  constexpr int TGPLK = (HALFN ? 64 : 128) * TP;  // G rows staged (HALFN: Nr <= 64)
  __shared__ __attribute__((aligned(16))) uint16_t Gt[2][NPL * TGPLK];
  __shared__ __attribute__((aligned(16))) uint16_t At[2][APN * TAPLK];
  __shared__ float scan_red[2 * (TX_THREADS / 64)];
  __shared__ float Ps[MAXPROJ * 128];
  __shared__ float dzL[2][TX_THREADS];  // rows 0..63 used; all threads write (branch-free staging)
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ntile = HALFN ? (wave & 1) : wave;
  const int t0 = HALFN ? (wave >> 1) * KT : 0;  // first k-tile of this wave
  const int Kc = a.k1 + a.k2;
  const int nkt = (Kc + 31) / 32;
  const int KP = nkt * 32;
  const int64_t mbeg = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t mend = min(a.M, mbeg + a.rows_per_block);
  const int nch = mend > mbeg ? (int)((mend - mbeg + TMC - 1) / TMC) : 0;

  floatx16 acc[KT];  // KT >= nkt k-tiles, computed unconditionally (tiles >= nkt are discarded)
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  if constexpr (PROJ) {
    if (tid < 128) {
#pragma unroll
      for (int q = 0; q < MAXPROJ; ++q) Ps[q * 128 + tid] = (q < a.nproj && tid < a.Nr) ? a.proj[q * a.Nr + tid] : 0.0f;
    }
  }

  // ---- slot descriptors
  const int gn = tid & 127, go = tid >> 7;
  const bool gcol = gn < a.Nr;
  const int gnc = gcol ? gn : 0;
  const float* base[NS];
  int ld32[NS];
  int oct[NS];
  int ak[TX_AS];
  bool aon[TX_AS];
#pragma unroll
  for (int sl = 0; sl < TX_AS; ++sl) {
    const int u = tid + TX_THREADS * sl;
    aon[sl] = u < 2 * KP;
    // idle slots stage nothing (their loads read a fixed address; the LDS columns they would fill
    // are only read by tiles t >= nkt, whose dW is discarded)
    ak[sl] = aon[sl] ? u % KP : 0;
    oct[sl] = aon[sl] ? u / KP : 0;
    const int k = ak[sl];
    if (aon[sl] && k < a.k1) { base[sl] = elem_ptr<ABF>(a.a1, k); ld32[sl] = (int)a.lda1; }
    else if (aon[sl] && k < Kc) { base[sl] = elem_ptr<ABF>(a.a2, k - a.k1); ld32[sl] = (int)a.lda2; }
    else { base[sl] = a.a1; ld32[sl] = 0; }
  }
  if constexpr (MASK) { base[GS] = elem_ptr<HBF>(a.h, gnc); ld32[GS] = (int)a.ldh; }
  else { base[GS] = a.g + gnc; ld32[GS] = (int)a.ldg; }
  oct[GS] = go;
  if constexpr (NS == GS + 2) { base[GS + 1] = a.g + gnc; ld32[GS + 1] = (int)a.ldg; oct[GS + 1] = go; }
  // dz element of this thread (threads 0..63 keep theirs: row tid/4, column tid%4)
  const int zr = (tid & 63) / MAXPROJ, zq = (tid & 63) % MAXPROJ;
  const int zqc = PROJ ? min(zq, a.nproj - 1) : 0;

  // 32-bit element offsets (the dispatcher guarantees M·ld < 2^31): rows clamped to mend - 1
  // Chunk c covers rows [mbeg + 16c, +16) but is LOADED from row ldbase(c) = min(that, M - 16)
  // (the dispatcher guarantees M >= 16): every load is in bounds with no per-element clamp,
  // rows past mend belong to the next block or repeat earlier rows, and the G mask (rows
  // [lo, hi) of the loaded chunk) zeroes them.
  const int Mi = (int)a.M;
  auto ldbase = [&](int c) { return min((int)mbeg + c * TMC, Mi - TMC); };
  float rv[D][NS][8];
  float rz[D];
  auto load = [&](int d, int c) {
    const int mb = ldbase(c);
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
      uint32_t o = (uint32_t)((mb + 8 * oct[sl]) * ld32[sl]);  // one multiply per slot (rows by adds)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t off = o;
        o += (uint32_t)ld32[sl];
        const bool bf = sl < TX_AS ? ABF : (sl == GS && MASK ? HBF : false);  // compile-time per slot
        rv[d][sl][i] = bf ? bf16_to_f32(reinterpret_cast<const uint16_t*>(base[sl])[off]) : base[sl][off];
      }
    }
    if constexpr (PROJ) {  // dz rows of chunk c + 1
      rz[d] = a.dz[(uint32_t)((ldbase(c + 1) + zr) * (int)a.lddz + zqc)];
    }
  };

  float db = 0.f, dzs = 0.f;
  float dw2[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  float sa = 1.f, sg = 1.f, una = 1.f, ung = 1.f;  // H2S: the block's A / G scales and their inverses
  auto put8 = [](uint16_t* dst, int plane, const float (&e)[8]) {
    uint32_t w[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) split_pair(e[2 * j], e[2 * j + 1], w[j]);
#pragma unroll
    for (int p = 0; p < NPL; ++p)
      *reinterpret_cast<uint4*>(dst + p * plane) = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
  };
  // H2S: 8 values times the scale s as half-pair planes — NP = 2: hi, lo (A); NP = 3: hi', hi, lo (G)
  auto put8h = [](uint16_t* dst, int plane, const float (&e)[8], float sc, auto npc) {
    constexpr int NP = decltype(npc)::value;
    uint32_t w[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t hi, lo;
      split_h2_pair(e[2 * j] * sc, e[2 * j + 1] * sc, hi, lo);
      if constexpr (NP == 3) { w[j][0] = h2_scale_pair(hi, 2048.0f); w[j][1] = hi; w[j][2] = lo; }
      else { w[j][0] = hi; w[j][1] = lo; }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p)
      *reinterpret_cast<uint4*>(dst + p * plane) = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
  };
  auto store = [&](int d, int c) {
    const int buf = c & 1;
    const int mb = ldbase(c);
    const int rlo = (int)mbeg + c * TMC - mb;  // valid loaded rows: [rlo, rhi)
    const int rhi = (int)mend - mb;
    if constexpr (PROJ) {  // slot read by G(c - 1), behind barrier c - 1 (threads >= 64: unused)
      const int mb1 = ldbase(c + 1);
      const bool ok = tid < TMC * MAXPROJ && zq < a.nproj && zr >= (int)mbeg + (c + 1) * TMC - mb1 &&
                      zr < (int)mend - mb1;
      dzL[(c + 1) & 1][tid] = ok ? rz[d] : 0.0f;
    }
    // A is stored unmasked: rows past mend were loaded clamped (finite copies of the last row)
    // and meet G = 0 there; columns >= Kc (padding, idle slots at KMAX - 1) only feed dW
    // columns that are never written out
#pragma unroll
    for (int sl = 0; sl < TX_AS; ++sl) {
      if (!aon[sl]) continue;  // (LDS stores only: the loads above stay unconditional)
      if constexpr (H2S) put8h(At[buf] + ak[sl] * TP + 8 * oct[sl], TAPLK, rv[d][sl], sa, std::integral_constant<int, 2>{});
      else put8(At[buf] + ak[sl] * TP + 8 * oct[sl], TAPLK, rv[d][sl]);
    }
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 8 * go + i;
      const bool rok = r >= rlo && r < rhi;
      const bool ok = rok && gcol;
      float g;
      if constexpr (PROJ) {
        const float* z = &dzL[buf][r * MAXPROJ];
        g = z[0] * Ps[gn];
#pragma unroll
        for (int q = 1; q < MAXPROJ; ++q) g = fmaf(z[q], Ps[q * 128 + gn], g);
        // the staged dz rows are zero outside [rlo, rhi) (and P columns >= Nr are zero), so G,
        // dzᵀh and Σdz need no per-row masks here (h of those rows is finite: our activations)
        if constexpr (MASK) {
#pragma unroll
          for (int q = 0; q < MAXPROJ; ++q) dw2[q] = fmaf(z[q], rv[d][GS][i], dw2[q]);
        }
        if (gn < MAXPROJ) dzs += z[gn & (MAXPROJ - 1)];
      } else {
        g = rv[d][NS - 1][i];
      }
      if constexpr (MASK) g = rv[d][GS][i] > 0.0f ? g * a.hscale : 0.0f;
      if constexpr (!PROJ) g = ok ? g : 0.0f;
      db += g;
      if constexpr (GOUT) {
        if (a.gout && ok) a.gout[(int64_t)(mb + r) * a.ldgout + gn] = g;
      }
      e[i] = g;
    }
    if (HALFN && gn >= 64) return;  // (zero G columns past Nr <= 64: not staged)
    if constexpr (H2S) put8h(Gt[buf] + gn * TP + 8 * go, TGPLK, e, sg, std::integral_constant<int, 3>{});
    else put8(Gt[buf] + gn * TP + 8 * go, TGPLK, e);
  };

  const int fr = (lane & 31) * TP + 8 * (lane >> 5);
  auto compute = [&](int c) {
    const int buf = c & 1;
    if constexpr (H2S) {  // G: hi', hi, lo; A: hi, lo
      f16x8 gf[3], af[2][2];
#pragma unroll
      for (int p = 0; p < 3; ++p) gf[p] = lds_frag16(Gt[buf] + p * TGPLK + ntile * 32 * TP + fr);
#pragma unroll
      for (int p = 0; p < 2; ++p) af[0][p] = lds_frag16(At[buf] + p * TAPLK + t0 * 32 * TP + fr);
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        if (t + 1 < KT) {
#pragma unroll
          for (int p = 0; p < 2; ++p) af[(t + 1) & 1][p] = lds_frag16(At[buf] + p * TAPLK + (t0 + t + 1) * 32 * TP + fr);
        }
        // G_lo·A_hi + G_hi·A_lo + G_hi'·A_hi
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(gf[2], af[t & 1][0], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(gf[1], af[t & 1][1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(gf[0], af[t & 1][0], acc[t], 0, 0, 0);
      }
      return;
    }
    // software-pipelined: tile t+1's fragments are read before tile t's MFMAs issue, so with one
    // wave per SIMD the LDS latency hides behind the MFMAs instead of stalling every tile
    bf16x8 gf[NPL], af[2][NPL];
#pragma unroll
    for (int p = 0; p < NPL; ++p) gf[p] = lds_frag(Gt[buf] + p * TGPLK + ntile * 32 * TP + fr);
#pragma unroll
    for (int p = 0; p < NPL; ++p) af[0][p] = lds_frag(At[buf] + p * TAPLK + t0 * 32 * TP + fr);
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if (t + 1 < KT) {
#pragma unroll
        for (int p = 0; p < NPL; ++p) af[(t + 1) & 1][p] = lds_frag(At[buf] + p * TAPLK + (t0 + t + 1) * 32 * TP + fr);
      }
      acc[t] = mfma_planes<NPL>(gf, af[t & 1], acc[t]);
    }
  };

  auto prologue = [&]() {
    if constexpr (PROJ) {  // dz of chunk 0
      const int mb0 = ldbase(0);
      const bool ok0 = tid < TMC * MAXPROJ && zq < a.nproj && zr >= (int)mbeg - mb0 && zr < (int)mend - mb0;
      dzL[0][tid] = ok0 ? a.dz[(int64_t)(mb0 + zr) * a.lddz + zqc] : 0.0f;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) load(d, min(d, nch - 1));
    if constexpr (H2S) {  // the block's bounds (behind chunk 0's loads): max row_exp, max |g|
      // A: every row a chunk loads — from ldbase(0) = min(mbeg, M - 16), so a last block of < 16
      // rows also bounds the earlier rows its clamped chunk re-reads (they meet G = 0, but an
      // unbounded A there would overflow f16 and turn 0 · inf into NaN)
      int ea = 0;
      for (int64_t r = ldbase(0) + tid; r < mend; r += TX_THREADS) ea = max(ea, a.rowexp[r]);
      float gm = 0.f;
      const int n4 = a.Nr >> 2;
      const int64_t npc = (mend - mbeg) * n4;
      constexpr int SU = 8;
      for (int64_t q0 = tid; q0 < npc; q0 += SU * TX_THREADS) {
        float4 v[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int64_t q = min(q0 + (int64_t)TX_THREADS * u, npc - 1);
          const int64_t r = mbeg + q / n4;
          v[u] = *reinterpret_cast<const float4*>(a.g + r * a.ldg + (q - (q / n4) * n4) * 4);
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const float m = fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w)));
          gm = fmaxf(gm, q0 + (int64_t)TX_THREADS * u < npc ? m : 0.f);
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        ea = max(ea, __shfl_xor(ea, o));
        gm = fmaxf(gm, __shfl_xor(gm, o));
      }
      if (lane == 0) {
        scan_red[wave] = __int_as_float(ea);
        scan_red[TX_THREADS / 64 + wave] = gm;
      }
    }
  };
  auto finish_scales = [&]() {  // after the prologue's barrier
    if constexpr (H2S) {
      int ea = __float_as_int(scan_red[0]);
      float gm = scan_red[TX_THREADS / 64];
#pragma unroll
      for (int w = 1; w < TX_THREADS / 64; ++w) {
        ea = max(ea, __float_as_int(scan_red[w]));
        gm = fmaxf(gm, scan_red[TX_THREADS / 64 + w]);
      }
      const int eg = h2_row_exp(gm);
      ea = min(ea, 127);
      sa = ldexpf(1.0f, 14 - ea);
      una = ldexpf(1.0f, ea - 14);
      sg = eg == 128 ? 1.0f : ldexpf(1.0f, 4 - eg);  // |G · sg| < 16
      ung = eg == 128 ? 1.0f / 2048.0f : ldexpf(1.0f, eg - 4 - 11);
    }
  };

  // ---- this block's partial dW (segment-major: dW1 = [Nr][k1] then dW2 = [Nr][k2])
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride;
  auto write_slab = [&]() {
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if (t0 + t >= nkt) continue;
      const int col = (t0 + t) * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = ntile * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int64_t idx = col < a.k1 ? (int64_t)row * a.k1 + col
                                       : (int64_t)a.Nr * a.k1 + (int64_t)row * a.k2 + (col - a.k1);
        if (row < a.Nr && col < Kc) slab[idx] = H2S ? (acc[t][r] * una) * ung : acc[t][r];
      }
    }
  };
  // ---- side sums of the two row octets (G slots, threads < 256), combined in a fixed order via
  //      LDS (At[0], free once every MFMA has read it: the caller's barrier)
  float* red = reinterpret_cast<float*>(&At[0][0]);
  constexpr int ns = 2 + MAXPROJ;
  auto side_put = [&]() {
    red[(go * 128 + gn) * ns + 0] = db;
    red[(go * 128 + gn) * ns + 1] = dzs;
#pragma unroll
    for (int q = 0; q < MAXPROJ; ++q) red[(go * 128 + gn) * ns + 2 + q] = dw2[q];
  };
  auto side_write = [&]() {
    if (tid < 128 && tid < a.Nr) {
      float* side = slab + (int64_t)a.Nr * Kc;
      side[tid] = red[tid * ns] + red[(128 + tid) * ns];
      for (int q = 0; q < a.nproj; ++q)
        side[a.Nr + q * a.Nr + tid] = red[tid * ns + 2 + q] + red[(128 + tid) * ns + 2 + q];
    }
    if (PROJ && tid < a.nproj)
      slab[(int64_t)a.Nr * Kc + a.Nr + a.nproj * a.Nr + tid] = red[tid * ns + 1] + red[(128 + tid) * ns + 1];
  };

  if (nch > 0) {
    prologue();
    __syncthreads();  // Ps, dzL[0] (H2S: the scan partials)
    finish_scales();
    if constexpr (PIPE != 0) {
      // software-pipelined order: between two barriers, chunk c+1 is staged into the other
      // buffers while chunk c's MFMAs run (PIPE == 2 adds interleave hints for the scheduler)
      store(0, 0);
      load(0, min(D, nch - 1));
      int c = 0;
      for (; c + D < nch; c += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const int cc = c + d;
          const int d1 = (d + 1) % D;
          __syncthreads();
          store(d1, cc + 1);
          load(d1, min(cc + 1 + D, nch - 1));
          compute(cc);
          if constexpr (PIPE == 2) {
#pragma unroll
            for (int i = 0; i < KT * (NPL == 3 ? 6 : 1); ++i) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
              __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // VALU
              __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
            }
          }
        }
      }
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int cc = c + d;
        if (cc < nch) {
          __syncthreads();
          if (cc + 1 < nch) store((d + 1) % D, cc + 1);
          compute(cc);
        }
      }
    } else {
    int c0 = 0;
    for (; c0 + D <= nch; c0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int c = c0 + d;
        store(d, c);  // buffers of chunk c - 2: last read before barrier c - 1
        __syncthreads();
        load(d, min(c + D, nch - 1));
        compute(c);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int c = c0 + d;
      if (c < nch) {
        store(d, c);
        __syncthreads();
        compute(c);
      }
    }
    }
  }

  write_slab();
  __syncthreads();
  side_put();
  __syncthreads();
  side_write();
}

// the split-bf16 TN (NPL = 3: 6 products; NPL = 1: the bf16-storage form) and its in-kernel
// half-pair form (GNN_MATH_HALF_PAIR), one body, two kernel names
template <bool PROJ, bool MASK, int D, int KT, int NPL = 3, bool ABF = false, bool HBF = false, int PIPE = 0,
          bool GOUT = true, bool HALFN = false>
__global__ __launch_bounds__(TX_THREADS) void gemm_tn_x3_kernel(TNArgs a) {
  gemm_tn_split_body<PROJ, MASK, D, KT, NPL, ABF, HBF, PIPE, GOUT, HALFN, false>(a);
}
template <int KT, bool HALFN>
__global__ __launch_bounds__(TX_THREADS) void gemm_tn_h2s_kernel(TNArgs a) {
  gemm_tn_split_body<false, false, 1, KT, 3, false, false, 0, false, HALFN, true>(a);
}

}  // namespace

size_t nt_x3_workspace(int64_t k1, int64_t k2) {  // pre-split B image, 12 KB per 16-deep chunk
  // (segments padded to 32-deep chunks), + 64 B of zeros; the weight-stationary form also keeps
  // its zero-padded tail tile here ([32][k1 + k2] f32 after its B image)
  const size_t x3 = (size_t)(2 * ((k1 + 31) / 32) + 2 * ((k2 + 31) / 32)) * 3 * 256 * sizeof(uint4) + 64;
  const size_t ws = nt_ws_tail_offset(k1, k2) + (size_t)32 * (k1 + k2) * sizeof(float);
  return x3 > ws ? x3 : ws;
}

void launch_nt_x3(const NTArgs& a, void* ws, size_t ws_bytes, hipStream_t st) {
  auto al = [](const void* q, int b) { return (reinterpret_cast<uintptr_t>(q) % b) == 0; };
  auto av_ok = [&](int v) {
    return (a.k1 % v == 0) && (a.lda1 % v == 0) && al(a.a1, 4 * v) &&
           (a.k2 == 0 || ((a.k2 % v == 0) && (a.lda2 % v == 0) && al(a.a2, 4 * v)));
  };
  const uint4* bimg = nullptr;
  if (a.a_bf16) {  // bf16 storage: one product per MFMA on bf16 operands (B rounded to bf16)
    auto bv_ok = [&](int v) {
      return (a.k1 % v == 0) && (a.lda1 % v == 0) && al(a.a1, 2 * v) &&
             (a.k2 == 0 || ((a.k2 % v == 0) && (a.lda2 % v == 0) && al(a.a2, 2 * v)));
    };
    const bool pre = ws && ws_bytes >= nt_x3_workspace(a.k1, a.k2) && a.Nc <= BN;
    if (pre) {
      const int nch1 = (a.k1 + 15) / 16, nch = nch1 + (a.k2 + 15) / 16;
      x3_presplit_b_kernel<<<nch, 256, 0, st>>>(a, static_cast<uint4*>(ws), nch1, nch);
      bimg = static_cast<const uint4*>(ws);
    }
    dim3 grid((unsigned)ceil_div(a.M, 128), (unsigned)ceil_div(a.Nc, BN));
#define GNN_NTB(AVV, BVV, C) gemm_nt_x3_kernel<16, 1, AVV, 2, BVV, 2, 1, true, C, BVV == 0 ? NT_PIPE | NT_HINTS : 0><<<grid, 256, 0, st>>>(a, bimg)
#define GNN_NTB_C(AVV, BVV) do { if (a.c_bf16) GNN_NTB(AVV, BVV, true); else GNN_NTB(AVV, BVV, false); } while (0)
    const bool v2 = bv_ok(2);
    if (bimg) { if (v2) GNN_NTB_C(2, 0); else GNN_NTB_C(1, 0); }
    else if (a.wvec >= 2) { if (v2) GNN_NTB_C(2, 2); else GNN_NTB_C(1, 2); }
    else { if (v2) GNN_NTB_C(2, 1); else GNN_NTB_C(1, 1); }
#undef GNN_NTB_C
#undef GNN_NTB
    return;
  }
  const int av = av_ok(4) ? 4 : (av_ok(2) ? 2 : 1);
  const bool pre = ws && ws_bytes >= nt_x3_workspace(a.k1, a.k2) && a.Nc <= BN;
  if (pre && nt_ws_ok(a)) {
    // the weight-stationary persistent form (gemm_ws.hip, its own B image in `ws`)
    launch_nt_ws(a, static_cast<uint4*>(ws), st);
    return;
  }
  if (pre) {
    const int nch1 = (a.k1 + 15) / 16, nch = nch1 + (a.k2 + 15) / 16;
    x3_presplit_b_kernel<<<nch, 256, 0, st>>>(a, static_cast<uint4*>(ws), nch1, nch);
    bimg = static_cast<const uint4*>(ws);
  }
  // The classic order (stage c; barrier; MFMAs of c) for the shapes outside nt_ws_ok.  r05-r10 lab
  // (Elliptic layer-1 shape): pipelined order + sched_group_barrier interleave 155-159 us vs
  // classic 171-182; D = 1 / 3 ring 228 / 188; A fragments straight to registers 291; an LDS-DMA
  // form 151-167; TM = 2 216-233 — the weight-stationary form (135 us) replaced them.
  launch_nt_x3_a<16, 1, 2, 2>(a, av, bimg, st);
}

template <int D, int KT, int NPL = 3, bool ABF = false, bool HBF = false, int PIPE = 0, bool GO = false,
          bool HN = false>
void launch_tn_x3_kg(const TNArgs& a, int nblk, hipStream_t st) {
  const bool proj = a.dz != nullptr, mask = a.h != nullptr;
  if (proj && mask) gemm_tn_x3_kernel<true, true, D, KT, NPL, ABF, HBF, PIPE, GO, HN><<<nblk, TX_THREADS, 0, st>>>(a);
  else if (proj) gemm_tn_x3_kernel<true, false, D, KT, NPL, ABF, HBF, PIPE, GO, HN><<<nblk, TX_THREADS, 0, st>>>(a);
  else if (mask) gemm_tn_x3_kernel<false, true, D, KT, NPL, ABF, HBF, PIPE, GO, HN><<<nblk, TX_THREADS, 0, st>>>(a);
  else gemm_tn_x3_kernel<false, false, D, KT, NPL, ABF, HBF, PIPE, GO, HN><<<nblk, TX_THREADS, 0, st>>>(a);
}

// the G write-out (gout, needed only when a further layer's dh follows) is a compile-time branch
template <int D, int KT, int NPL = 3, bool ABF = false, bool HBF = false, int PIPE = 0, bool HN = false>
void launch_tn_x3_k(const TNArgs& a, int nblk, hipStream_t st) {
  if (a.gout) launch_tn_x3_kg<D, KT, NPL, ABF, HBF, PIPE, true, HN>(a, nblk, st);
  else launch_tn_x3_kg<D, KT, NPL, ABF, HBF, PIPE, false, HN>(a, nblk, st);
}


// Lab (MI355X, Elliptic layer-1 TN, dz form + mask, variants interleaved in one process): with the
// staging VALU cut from ~530 to ~325 per chunk (unmasked A, row offsets by adds, no per-row masks
// in the dz form) the classic order runs 156 us and the pipelined order with interleave hints
// 183 (before the cuts: 207 vs 196).  A 32-row-chunk variant measured 217-227 and was removed.
// r08 (removed after measuring): a deeper load ring D = 2 / 3 in the classic order 166 / 159 us
// vs 156; a wave-specialised form (512 threads: 4 producer waves stage chunk c + 1 while 4
// consumer waves run chunk c's MFMAs, one barrier per chunk, 218-230 VGPRs, no spills) 150 / 148
// (D = 1 / 2) vs 153 — no overlap materialised.  PMC of the production kernel per wave and
// 16-row chunk (6,080 cycles): ~420 VALU (1,700 issue cycles: split ~265, load addressing ~95),
// 66 MFMAs (2,112 cycles), waits at s_waitcnt / barrier ~1,560 — the VALU and MFMA phases add.
// Further r09 forms, all correct vs float64 and all removed: a fenced interleave (chunk k+1 staged
// in ~20 units placed between chunk k's MFMAs by sched_barrier fences, 2-deep ring, loads issued
// right after each slot is consumed) 150-155 us; its ablations: no MFMAs 103, L2-hot loads 153
// (not HBM-bound); two waves per SIMD (512 threads, half the k-tiles per wave, 2 A slots + a
// 4-row G slot per thread) 164.  Every form lands at ~6,000 cycles per chunk per SIMD.
void launch_tn_x3(const TNArgs& a, int nblk, hipStream_t st) {
  const int nkt = (a.k1 + a.k2 + 31) / 32;
  constexpr int D = 1;
  if (a.a_bf16) {
    if (nkt <= 8) { if (a.h_bf16) launch_tn_x3_k<D, 8, 1, true, true, 0>(a, nblk, st); else launch_tn_x3_k<D, 8, 1, true, false, 0>(a, nblk, st); }
    else { if (a.h_bf16) launch_tn_x3_k<D, 12, 1, true, true, 0>(a, nblk, st); else launch_tn_x3_k<D, 12, 1, true, false, 0>(a, nblk, st); }
    return;
  }
  // production: classic order (stage c; barrier; MFMAs of c).  Nr <= 64 (GCN / GAT / SAGE-ResBN
  // hidden width 64): the half-N mapping, ceil(nkt / 2) k-tiles per wave
  if (a.Nr <= 64) {
    const int kh = (nkt + 1) / 2;
    if (kh <= 2) launch_tn_x3_k<D, 2, 3, false, false, 0, true>(a, nblk, st);
    else if (kh <= 3) launch_tn_x3_k<D, 3, 3, false, false, 0, true>(a, nblk, st);
    else if (kh <= 4) launch_tn_x3_k<D, 4, 3, false, false, 0, true>(a, nblk, st);
    else launch_tn_x3_k<D, 6, 3, false, false, 0, true>(a, nblk, st);
    return;
  }
  if (nkt <= 6) launch_tn_x3_k<D, 6, 3, false, false, 0>(a, nblk, st);
  else if (nkt <= 8) launch_tn_x3_k<D, 8, 3, false, false, 0>(a, nblk, st);
  else if (nkt <= 11) launch_tn_x3_k<D, 11, 3, false, false, 0>(a, nblk, st);
  else launch_tn_x3_k<D, 12, 3, false, false, 0>(a, nblk, st);
}

// ---- the in-kernel half-pair forms (GNN_MATH_HALF_PAIR)
bool nt_h2s_ok(const NTArgs& a) {
  return !a.a_bf16 && !a.c_bf16 && a.w1 && !a.bt && a.Nc >= 1 && a.Nc <= BN && a.k1 % 16 == 0 && a.k2 % 16 == 0 &&
         a.k1 + a.k2 >= 16 && a.k1 + a.k2 <= 128 && (a.k2 == 0 || a.w2) && !a.mask;
}

size_t nt_h2s_workspace(int64_t k1, int64_t k2) {  // the half-pair B image + BN column scales
  return (size_t)(k1 / 16 + k2 / 16) * 3 * 256 * sizeof(uint4) + BN * sizeof(float);
}

void launch_nt_h2s(const NTArgs& a, void* ws, hipStream_t st) {
  const int nch1 = a.k1 / 16, nch = nch1 + a.k2 / 16;
  H2Prep p{};
  p.w1 = a.w1; p.w2 = a.w2; p.ldw1 = a.ldw1; p.ldw2 = a.ldw2;
  p.k1 = a.k1; p.k2 = a.k2; p.Nc = a.Nc; p.col2 = 16 * nch1;  // chunk c = k-step c
  p.blocks = nch;
  p.img = static_cast<uint4*>(ws);
  p.colscale = reinterpret_cast<float*>(p.img + (size_t)nch * 3 * 256);
  p.a_unscale = 1.0f;  // (the A scales are per row, undone in the kernel's epilogue)
  launch_prep_h2(p, st);
  auto al = [](const void* q, int b) { return (reinterpret_cast<uintptr_t>(q) % b) == 0; };
  const bool v4 = (a.lda1 % 4 == 0) && al(a.a1, 16) && (a.k2 == 0 || ((a.lda2 % 4 == 0) && al(a.a2, 16)));
  const bool v2 = (a.lda1 % 2 == 0) && al(a.a1, 8) && (a.k2 == 0 || ((a.lda2 % 2 == 0) && al(a.a2, 8)));
  const dim3 grid((unsigned)ceil_div(a.M, 128));
  const uint4* img = p.img;
#define GNN_H2S_V(NCHV, NTLV)                                                                  \
  do {                                                                                         \
    if (v4) gemm_nt_h2s_kernel<NCHV, NTLV, 4><<<grid, 256, 0, st>>>(a, img);                  \
    else if (v2) gemm_nt_h2s_kernel<NCHV, NTLV, 2><<<grid, 256, 0, st>>>(a, img);             \
    else gemm_nt_h2s_kernel<NCHV, NTLV, 1><<<grid, 256, 0, st>>>(a, img);                     \
  } while (0)
#define GNN_H2S_N(NCHV) do { if (a.Nc <= 64) GNN_H2S_V(NCHV, 2); else GNN_H2S_V(NCHV, 4); } while (0)
  switch (nch) {  // (nt_h2s_ok: 1 <= nch <= 8)
    case 1: GNN_H2S_N(1); break;
    case 2: GNN_H2S_N(2); break;
    case 3: GNN_H2S_N(3); break;
    case 4: GNN_H2S_N(4); break;
    case 5: GNN_H2S_N(5); break;
    case 6: GNN_H2S_N(6); break;
    case 7: GNN_H2S_N(7); break;
    default: GNN_H2S_N(8); break;
  }
#undef GNN_H2S_N
#undef GNN_H2S_V
}

bool tn_h2s_ok(const TNArgs& a) {
  auto al = [](const void* q, int b) { return (reinterpret_cast<uintptr_t>(q) % b) == 0; };
  return a.rowexp && !a.dz && !a.h && !a.gout && a.g && !a.a_bf16 && !a.g_bf16 && a.Nr % 4 == 0 && a.Nr <= 128 &&
         a.ldg % 4 == 0 && al(a.g, 16) && a.k1 + a.k2 <= KMAX && a.M >= 16;
}

void launch_tn_h2s(const TNArgs& a, int nblk, hipStream_t st) {
  const int nkt = (a.k1 + a.k2 + 31) / 32;
#define GNN_TNH(KTV, HN) gemm_tn_h2s_kernel<KTV, HN><<<nblk, TX_THREADS, 0, st>>>(a)
  if (a.Nr <= 64) {  // the half-N mapping (as launch_tn_x3)
    const int kh = (nkt + 1) / 2;
    if (kh <= 2) GNN_TNH(2, true);
    else if (kh <= 3) GNN_TNH(3, true);
    else if (kh <= 4) GNN_TNH(4, true);
    else GNN_TNH(6, true);
  } else if (nkt <= 6) GNN_TNH(6, false);
  else if (nkt <= 8) GNN_TNH(8, false);
  else if (nkt <= 11) GNN_TNH(11, false);
  else GNN_TNH(12, false);
#undef GNN_TNH
}

}  // namespace gnnmp
