// K7 — fp32 MFMA GEMMs for the dense transforms of SAGEConv/GCNConv/GATConv, with the
// surrounding elementwise work of src/models/gnn.py fused in.
//
// Replaces PyG Linear (lin_l / lin_r / lin, gnn.py:41-44, 20-23, 64-67) and the ReLU +
// dropout between layers (gnn.py:29-30, 50-51) — forward (NT kernel) and weight
// gradients (TN kernel).  Exact fp32: v_mfma_f32_32x32x2_f32 is a k-ordered fmaf chain
// (no TF32/xf32 on gfx950), so results are within fp32 rounding of ATen's sgemm.
//
// NT:  C[M,Nc] = epi( [A1 | A2][M, k1+k2] · Bt[k1+k2, Nc] )
//      epi = +bias, ReLU, dropout (counter hash, keep prob 1-p, scale 1/(1-p)),
//      optional projection Z[M,nproj] = C · Pᵀ (P [nproj, Nc]) — the next, narrow layer's
//      transform-first GEMM computed from registers (the hidden activations' row is whole
//      in one wave).  Block = 4 waves x (32 rows x 128 cols); K streamed in 32-deep chunks
//      through double-buffered LDS (A padded to 33 floats/row: conflict-free b32 reads).
// TN:  dW[Nr, k1+k2] = Σ_m G[m, Nr]ᵀ · [A1 | A2][m, :]   (split over M, slabs, ordered reduce)
//      G = (G_src or dz·P) ⊙ (h > 0 ? scale : 0)   — ReLU+dropout backward computed on the fly
//      side sums: db[n] = Σ G, dW2[q][n] = Σ dz[m,q]·h[m,n], dzsum[q] = Σ dz[m,q]
//      Block = 16 waves: wave w owns dW rows (w&3)*32.. and k-tiles (w>>2)*3 .. +3.
// Both are atomic-free and deterministic.
#include "common.hpp"

#include <algorithm>
#include <cstdlib>

#include "gemm_common.hpp"

namespace gnnmp {
namespace {

constexpr int BNP = BN + 2;  // LDS pitch of the B tile: 2P = 4 mod 32 makes the transposed weight stores (8 lanes x float2 per row) conflict-free


// Tiling parameters: KC = K depth per LDS chunk, TM = 32-row tiles per wave (block rows
// BM = 4 waves x 32·TM), UNR = fully unroll full chunks.
template <int KC, int TM>
struct NTShape {
  static constexpr int BM = 128 * TM;
  static constexpr int APITCH = KC + 1;  // odd pitch: conflict-free column reads of A
  static constexpr int A_PER_THREAD = BM * KC / 256;
  static constexpr int B_PER_THREAD = KC * BN / 256;
};

template <int KC>
__device__ __forceinline__ void nt_chunk_range(const NTArgs& a, int c, const float*& A, int64_t& lda, int& k0,
                                               int& kb0, int& klen) {
  const int nch1 = (a.k1 + KC - 1) / KC;
  if (c < nch1) { A = a.a1; lda = a.lda1; k0 = c * KC; kb0 = k0; klen = min(KC, a.k1 - k0); }
  else { A = a.a2; lda = a.lda2; k0 = (c - nch1) * KC; kb0 = a.k1 + k0; klen = min(KC, a.k2 - k0); }
}

// Loads only (every address clamped into range, no data-dependent selects), so the
// prefetch of chunk c+1 stays in flight across chunk c's MFMAs; masking happens in
// nt_store, after them.  AVEC divides k1 and k2, so a vector never straddles K's end.
template <int AVEC, int KC, int TM>
__device__ __forceinline__ void nt_load(const NTArgs& a, int c, int64_t m0, int n0, bool bvec4,
                                        float (&ra)[NTShape<KC, TM>::A_PER_THREAD],
                                        float (&rb)[NTShape<KC, TM>::B_PER_THREAD]) {
  using S = NTShape<KC, TM>;
  const float* A; int64_t lda; int k0, kb0, klen;
  nt_chunk_range<KC>(a, c, A, lda, k0, kb0, klen);
  constexpr int VPR = KC / AVEC;
#pragma unroll
  for (int i = 0; i < S::A_PER_THREAD / AVEC; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int r = v / VPR;
    const int k = (v % VPR) * AVEC;
    int64_t row = m0 + r;
    row = row < a.M ? row : a.M - 1;
    const float* p = A + row * lda + k0 + (k < klen ? k : 0);
    if constexpr (AVEC == 4) {
      float4 t = *reinterpret_cast<const float4*>(p);
      ra[i * 4 + 0] = t.x; ra[i * 4 + 1] = t.y; ra[i * 4 + 2] = t.z; ra[i * 4 + 3] = t.w;
    } else if constexpr (AVEC == 2) {
      float2 t = *reinterpret_cast<const float2*>(p);
      ra[i * 2 + 0] = t.x; ra[i * 2 + 1] = t.y;
    } else {
      ra[i] = *p;
    }
  }
  if (a.w1) {
    // B from PyTorch Linear weights W [Nc, K] read in place (no transposed copy): 8 lanes cover
    // KC consecutive k of one weight row with float2 loads (4·KC contiguous bytes).
    const bool seg1 = c < (a.k1 + KC - 1) / KC;
    const float* W = seg1 ? a.w1 : a.w2;
    const int64_t ldw = seg1 ? a.ldw1 : a.ldw2;
#pragma unroll
    for (int i = 0; i < S::B_PER_THREAD / 2; ++i) {
      const int v = threadIdx.x + 256 * i;  // float2 slots: 128 rows x KC/2
      const int n = v / (KC / 2);
      const int kk = (v % (KC / 2)) * 2;
      const int nn = n0 + n < a.Nc ? n0 + n : 0;
      const float* p = W + (int64_t)nn * ldw + k0 + (kk < klen ? kk : 0);
      if (a.wvec2) {
        float2 t = *reinterpret_cast<const float2*>(p);
        rb[2 * i] = t.x; rb[2 * i + 1] = t.y;
      } else {
        rb[2 * i] = p[0];
        rb[2 * i + 1] = p[kk + 1 < klen ? 1 : 0];
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < S::B_PER_THREAD / 4; ++i) {
    const int v = threadIdx.x + 256 * i;  // float4 slots: KC rows x 32
    const int kk = v >> 5;
    const int n = (v & 31) * 4;
    const float* p = a.bt + (int64_t)(kb0 + (kk < klen ? kk : 0)) * a.ldb;
    if (bvec4) {  // Nc % 4 == 0: a float4 never straddles Nc
      const int nn = n0 + n < a.Nc ? n0 + n : 0;
      float4 t = *reinterpret_cast<const float4*>(p + nn);
      rb[i * 4 + 0] = t.x; rb[i * 4 + 1] = t.y; rb[i * 4 + 2] = t.z; rb[i * 4 + 3] = t.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) rb[i * 4 + q] = p[n0 + n + q < a.Nc ? n0 + n + q : 0];
    }
  }
}

template <int AVEC, int KC, int TM>
__device__ __forceinline__ void nt_store(const NTArgs& a, int c, int64_t m0, int n0, float* As, float* Bs,
                                         const float (&ra)[NTShape<KC, TM>::A_PER_THREAD],
                                         const float (&rb)[NTShape<KC, TM>::B_PER_THREAD]) {
  using S = NTShape<KC, TM>;
  const float* A; int64_t lda; int k0, kb0, klen;
  nt_chunk_range<KC>(a, c, A, lda, k0, kb0, klen);
  constexpr int VPR = KC / AVEC;
#pragma unroll
  for (int i = 0; i < S::A_PER_THREAD / AVEC; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int r = v / VPR;
    const int k = (v % VPR) * AVEC;
    const bool ok = (m0 + r < a.M) && (k < klen);
#pragma unroll
    for (int q = 0; q < AVEC; ++q) As[r * S::APITCH + k + q] = ok ? ra[i * AVEC + q] : 0.0f;
  }
  if (a.w1) {
#pragma unroll
    for (int i = 0; i < S::B_PER_THREAD / 2; ++i) {
      const int v = threadIdx.x + 256 * i;
      const int n = v / (KC / 2);
      const int kk = (v % (KC / 2)) * 2;
      const bool nok = n0 + n < a.Nc;
      Bs[kk * BNP + n] = (nok && kk < klen) ? rb[2 * i] : 0.0f;
      Bs[(kk + 1) * BNP + n] = (nok && kk + 1 < klen) ? rb[2 * i + 1] : 0.0f;
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < S::B_PER_THREAD / 4; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int kk = v >> 5;
    const int n = (v & 31) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) Bs[kk * BNP + n + q] = (kk < klen && n0 + n + q < a.Nc) ? rb[i * 4 + q] : 0.0f;
  }
}

template <int KC>
__device__ __forceinline__ int nt_ksteps(const NTArgs& a, int c) {
  const float* A; int64_t lda; int k0, kb0, klen;
  nt_chunk_range<KC>(a, c, A, lda, k0, kb0, klen);
  return (klen + 1) >> 1;
}

template <int TM>
__device__ __forceinline__ void nt_kstep(floatx16 (&acc)[TM][4], const float* Aw, const float* Bw, int s, int apitch) {
  float af[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) af[tm] = Aw[tm * 32 * apitch + 2 * s];
  const float* b = Bw + 2 * s * BNP;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float bf = b[t * 32];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm], bf, acc[tm][t], 0, 0, 0);
  }
}


template <int AVEC, int KC, int TM, bool UNR, int EXP = 0>
__global__ __launch_bounds__(256) void gemm_nt_kernel(NTArgs a) {
  using S = NTShape<KC, TM>;
  __shared__ float As[2][S::BM * S::APITCH];
  __shared__ float Bs[2][KC * BNP];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * S::BM;
  const int n0 = blockIdx.y * BN;
  const int nchunks = (a.k1 + KC - 1) / KC + (a.k2 + KC - 1) / KC;
  const bool bvec4 = ((a.ldb & 3) == 0) && ((a.Nc & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.bt) & 15) == 0);

  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;
  floatx16 acc[TM][4];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][t][r] = 0.0f;

  float ra[S::A_PER_THREAD], rb[S::B_PER_THREAD];
  nt_load<AVEC, KC, TM>(a, 0, m0, n0, bvec4, ra, rb);
  nt_store<AVEC, KC, TM>(a, 0, m0, n0, As[0], Bs[0], ra, rb);
  __syncthreads();

  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    if (EXP != 1 && EXP != 3 && c + 1 < nchunks) nt_load<AVEC, KC, TM>(a, c + 1, m0, n0, bvec4, ra, rb);
    const float* Aw = As[buf] + (wave * 32 * TM + (lane & 31)) * S::APITCH + (lane >> 5);
    const float* Bw = Bs[buf] + (lane >> 5) * BNP + (lane & 31);
    const int ks = nt_ksteps<KC>(a, c);
    if (EXP == 2) {
    } else if (UNR && ks == KC / 2) {
#pragma unroll
      for (int s = 0; s < KC / 2; ++s) nt_kstep<TM>(acc, Aw, Bw, s, S::APITCH);
    } else {
      for (int s = 0; s < ks; ++s) nt_kstep<TM>(acc, Aw, Bw, s, S::APITCH);
    }
    if (EXP != 3 && c + 1 < nchunks) nt_store<AVEC, KC, TM>(a, c + 1, m0, n0, As[buf ^ 1], Bs[buf ^ 1], ra, rb);
    __syncthreads();
  }

  nt_epilogue<TM>(a, acc, m0, n0, lane, wave, seed);
}

template <int AVEC, int KC, int TM, bool UNR, int EXP = 0>
void launch_nt(const NTArgs& a, hipStream_t st) {
  dim3 grid((unsigned)ceil_div(a.M, NTShape<KC, TM>::BM), (unsigned)ceil_div(a.Nc, BN));
  gemm_nt_kernel<AVEC, KC, TM, UNR, EXP><<<grid, 256, 0, st>>>(a);
}

// ------------------------------------------------------------ NT, k-permuted b128 fragments
// Both LDS images are K-contiguous rows — A as [row][k], B as [n][k] (the PyTorch Linear weight
// layout, so W is staged in place) — with a pitch of KC+4 floats.  MFMA k-step j of k-group g
// pairs k = 8g+j (lanes 0-31) with k = 8g+4+j (lanes 32-63): each lane fetches the operands of
// four k-steps with ONE ds_read_b128 (pitch ≡ 20 or 36 mod 64 dwords keeps the b128 lane groups
// conflict-free), 5 LDS reads per 16 MFMAs instead of 20.  Every k is still summed exactly once
// per output, in a fixed order, with zero-filled tails in both operands.
template <int KC>
struct NT2Shape {
  static constexpr int BM = 128;
  static constexpr int P = KC + 4;
  static constexpr int A_PER_THREAD = BM * KC / 256;
  static constexpr int B_PER_THREAD = BN * KC / 256;
};

// Stage rows [r0, r0+128) x [k0, k0+KC) of a K-contiguous row-major operand into registers.
// Row and k are clamped (loads never depend on data: the prefetch stays in flight).
template <int VEC, int KC>
__device__ __forceinline__ void nt2_load_rows(const float* X, int64_t ldx, int64_t r0, int64_t rows, int k0,
                                              int klen, float* reg) {
  constexpr int VPR = KC / VEC;
#pragma unroll
  for (int i = 0; i < 128 * KC / 256 / VEC; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int r = v / VPR;
    const int k = (v % VPR) * VEC;
    int64_t row = r0 + r;
    row = row < rows ? row : rows - 1;
    const float* p = X + row * ldx + k0 + (k < klen ? k : 0);
    if constexpr (VEC == 4) {
      const float4 t = *reinterpret_cast<const float4*>(p);
      reg[i * 4 + 0] = t.x; reg[i * 4 + 1] = t.y; reg[i * 4 + 2] = t.z; reg[i * 4 + 3] = t.w;
    } else if constexpr (VEC == 2) {
      const float2 t = *reinterpret_cast<const float2*>(p);
      reg[i * 2 + 0] = t.x; reg[i * 2 + 1] = t.y;
    } else {
      reg[i] = *p;
    }
  }
}

template <int VEC, int KC>
__device__ __forceinline__ void nt2_store_rows(float* L, int64_t r0, int64_t rows, int klen, bool full,
                                               const float* reg) {
  constexpr int VPR = KC / VEC;
  constexpr int P = NT2Shape<KC>::P;
#pragma unroll
  for (int i = 0; i < 128 * KC / 256 / VEC; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int r = v / VPR;
    const int k = (v % VPR) * VEC;
    const bool ok = full || ((r0 + r < rows) && (k < klen));  // VEC divides klen: all-or-nothing
    float* d = L + r * P + k;
    if constexpr (VEC == 4) {
      *reinterpret_cast<float4*>(d) = ok ? make_float4(reg[i * 4], reg[i * 4 + 1], reg[i * 4 + 2], reg[i * 4 + 3])
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
    } else if constexpr (VEC == 2) {
      *reinterpret_cast<float2*>(d) = ok ? make_float2(reg[i * 2], reg[i * 2 + 1]) : make_float2(0.f, 0.f);
    } else {
      *d = ok ? reg[i] : 0.0f;
    }
  }
}

// B from the transposed copy Bt [K, Nc] (N-contiguous): lanes run along k so the transposed
// scalar LDS stores spread over the banks; k and n are clamped.
template <int KC>
__device__ __forceinline__ void nt2_load_bt(const NTArgs& a, int kb0, int klen, int n0, bool bvec4, float* reg) {
#pragma unroll
  for (int i = 0; i < BN * KC / 256 / 4; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int kk = v % KC;
    const int n = (v / KC) * 4;
    const float* p = a.bt + (int64_t)(kb0 + (kk < klen ? kk : 0)) * a.ldb;
    if (bvec4) {
      const int nn = n0 + n < a.Nc ? n0 + n : 0;
      const float4 t = *reinterpret_cast<const float4*>(p + nn);
      reg[i * 4 + 0] = t.x; reg[i * 4 + 1] = t.y; reg[i * 4 + 2] = t.z; reg[i * 4 + 3] = t.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) reg[i * 4 + q] = p[n0 + n + q < a.Nc ? n0 + n + q : 0];
    }
  }
}

template <int KC>
__device__ __forceinline__ void nt2_store_bt(const NTArgs& a, float* L, int klen, int n0, const float* reg) {
  constexpr int P = NT2Shape<KC>::P;
#pragma unroll
  for (int i = 0; i < BN * KC / 256 / 4; ++i) {
    const int v = threadIdx.x + 256 * i;
    const int kk = v % KC;
    const int n = (v / KC) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) L[(n + q) * P + kk] = (kk < klen && n0 + n + q < a.Nc) ? reg[i * 4 + q] : 0.0f;
  }
}

template <int AVEC, int BVEC, int KC, bool WFORM>
struct NT2Stage {
  using S = NT2Shape<KC>;
  float ra[S::A_PER_THREAD];
  float rb[S::B_PER_THREAD];
  __device__ __forceinline__ void load(const NTArgs& a, int c, int64_t m0, int n0, bool bvec4) {
    const float* A; int64_t lda; int k0, kb0, klen;
    nt_chunk_range<KC>(a, c, A, lda, k0, kb0, klen);
    nt2_load_rows<AVEC, KC>(A, lda, m0, a.M, k0, klen, ra);
    if constexpr (WFORM) {
      const bool seg1 = c < (a.k1 + KC - 1) / KC;
      nt2_load_rows<BVEC, KC>(seg1 ? a.w1 : a.w2, seg1 ? a.ldw1 : a.ldw2, n0, a.Nc, k0, klen, rb);
    } else {
      nt2_load_bt<KC>(a, kb0, klen, n0, bvec4, rb);
    }
  }
  __device__ __forceinline__ void store(const NTArgs& a, int c, int64_t m0, int n0, float* As, float* Bs) {
    const float* A; int64_t lda; int k0, kb0, klen;
    nt_chunk_range<KC>(a, c, A, lda, k0, kb0, klen);
    const bool kfull = klen == KC;
    nt2_store_rows<AVEC, KC>(As, m0, a.M, klen, kfull && m0 + S::BM <= a.M, ra);
    if constexpr (WFORM) nt2_store_rows<BVEC, KC>(Bs, n0, a.Nc, klen, kfull && n0 + BN <= a.Nc, rb);
    else nt2_store_bt<KC>(a, Bs, klen, n0, rb);
  }
};

template <int AVEC, int BVEC, int KC, bool WFORM, int EXP = 0, int DEPTH = 1>
__global__ __launch_bounds__(256) void gemm_nt2_kernel(NTArgs a) {
  using S = NT2Shape<KC>;
  constexpr int P = S::P;
  __shared__ __attribute__((aligned(16))) float As[2][S::BM * P];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * P];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * S::BM;
  const int n0 = blockIdx.y * BN;
  const int nch1 = (a.k1 + KC - 1) / KC;
  const int nchunks = nch1 + (a.k2 + KC - 1) / KC;
  const bool bvec4 = !WFORM && ((a.ldb & 3) == 0) && ((a.Nc & 3) == 0) &&
                     ((reinterpret_cast<uintptr_t>(a.bt) & 15) == 0);
  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;

  floatx16 acc[1][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][t][r] = 0.0f;

  const int foff = (lane & 31) * P + 4 * (lane >> 5);
  auto compute = [&](const float* Ab, const float* Bb, int c) {
    const int klen = c < nch1 ? min(KC, a.k1 - c * KC) : min(KC, a.k2 - (c - nch1) * KC);
    const int ng = (klen + 7) >> 3;
    const float* Af = Ab + wave * 32 * P + foff;
    const float* Bf = Bb + foff;
#pragma unroll
    for (int g = 0; g < KC / 8; ++g) {
      if (g < ng) {
        const float4 av = *reinterpret_cast<const float4*>(Af + 8 * g);
        float4 bv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) bv[t] = *reinterpret_cast<const float4*>(Bf + t * 32 * P + 8 * g);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv[t].x, acc[0][t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv[t].y, acc[0][t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv[t].z, acc[0][t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv[t].w, acc[0][t], 0, 0, 0);
      }
    }
  };

  if constexpr (DEPTH == 1) {
    NT2Stage<AVEC, BVEC, KC, WFORM> st;
    st.load(a, 0, m0, n0, bvec4);
    st.store(a, 0, m0, n0, As[0], Bs[0]);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
      const int buf = EXP >= 4 ? 0 : (c & 1);
      if ((EXP == 0 || EXP == 6) && c + 1 < nchunks) st.load(a, c + 1, m0, n0, bvec4);
      compute(As[buf], Bs[buf], c);
      if ((EXP == 0 || EXP == 7) && c + 1 < nchunks) st.store(a, c + 1, m0, n0, As[buf ^ 1], Bs[buf ^ 1]);
      if (EXP == 6 && c + 1 < nchunks) {  // keep the loads alive without the LDS stores
        float sink = 0.f;
#pragma unroll
        for (int i = 0; i < NT2Shape<KC>::A_PER_THREAD; ++i) sink += st.ra[i];
#pragma unroll
        for (int i = 0; i < NT2Shape<KC>::B_PER_THREAD; ++i) sink += st.rb[i];
        if (sink == 12345.678f) As[buf][threadIdx.x] = sink;
      }
      if (EXP != 4) __syncthreads();
    }
  } else {
    // Two register stages: while chunk c's MFMAs run, chunks c+1 and c+2 are in flight (one
    // chunk of MFMAs, ≈0.85 µs, is shorter than a loaded HBM round trip).
    NT2Stage<AVEC, BVEC, KC, WFORM> s0, s1;
    s0.load(a, 0, m0, n0, bvec4);
    s0.store(a, 0, m0, n0, As[0], Bs[0]);
    __syncthreads();
    if (1 < nchunks) s1.load(a, 1, m0, n0, bvec4);
    if (2 < nchunks) s0.load(a, 2, m0, n0, bvec4);
    for (int c = 0; c < nchunks; c += 2) {
      compute(As[0], Bs[0], c);
      if (c + 1 < nchunks) {
        s1.store(a, c + 1, m0, n0, As[1], Bs[1]);
        if (c + 3 < nchunks) s1.load(a, c + 3, m0, n0, bvec4);
      }
      __syncthreads();
      if (c + 1 >= nchunks) break;
      compute(As[1], Bs[1], c + 1);
      if (c + 2 < nchunks) {
        s0.store(a, c + 2, m0, n0, As[0], Bs[0]);
        if (c + 4 < nchunks) s0.load(a, c + 4, m0, n0, bvec4);
      }
      __syncthreads();
    }
  }
  nt_epilogue<1>(a, acc, m0, n0, lane, wave, seed);
}

template <int AVEC, int BVEC, int KC, bool WFORM, int EXP, int DEPTH>
void launch_nt2(const NTArgs& a, hipStream_t st) {
  dim3 grid((unsigned)ceil_div(a.M, NT2Shape<KC>::BM), (unsigned)ceil_div(a.Nc, BN));
  gemm_nt2_kernel<AVEC, BVEC, KC, WFORM, EXP, DEPTH><<<grid, 256, 0, st>>>(a);
}

template <int AVEC, int KC, int EXP = 0, int DEPTH = 1>
void launch_nt2_b(const NTArgs& a, hipStream_t st) {
  if (!a.w1) launch_nt2<AVEC, 1, KC, false, EXP, DEPTH>(a, st);
  else if (a.wvec == 4) launch_nt2<AVEC, 4, KC, true, EXP, DEPTH>(a, st);
  else if (a.wvec == 2) launch_nt2<AVEC, 2, KC, true, EXP, DEPTH>(a, st);
  else launch_nt2<AVEC, 1, KC, true, EXP, DEPTH>(a, st);
}

// The exact-f32 NT: 16-deep chunks, one chunk of loads in flight (r01 lab, the fastest of the
// [k][n]-image, 32-deep-chunk and two-chunks-in-flight forms).
template <int AVEC>
void launch_nt_f32(const NTArgs& a, hipStream_t st) {
  launch_nt2_b<AVEC, 16>(a, st);
}

// ------------------------------------------------------------------------------------ TN


// slab layout: dW[Nr][Kc] | db[Nr] | dW2[nproj][Nr] | dzsum[nproj]
//
// Structure (per 512-thread block, rows [mbeg, mend)): chunks of MC=32 rows, double-buffered
// through LDS.  While the MFMAs of chunk c run, chunk c+1's operands are already in flight
// into registers (every load unconditional on a clamped row: no branch-around-load waits);
// they are transformed (G prologue) and stored after the MFMAs, then one barrier.
template <int MC, int NTL>
__device__ __forceinline__ void tn_mma(floatx16 (&acc)[KT_PER_WAVE], const float* gptr, const float* aptr, int kt0) {
#pragma unroll 2
  for (int s = 0; s < MC / 2; ++s) {
    const float gf = gptr[2 * s * 128];
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
      const float af = aptr[2 * s * TN_APITCH + (kt0 + t) * 32];
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(gf, af, acc[t], 0, 0, 0);
    }
  }
}

template <bool PROJ, bool MASK, int AVEC, int MC>
__global__ __launch_bounds__(TN_THREADS) void gemm_tn_kernel(TNArgs a) {
  __shared__ __attribute__((aligned(16))) float Gs[2][MC * 128];
  __shared__ __attribute__((aligned(16))) float As[2][MC * TN_APITCH];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ntile = wave & 3;
  const int kt0 = (wave >> 2) * KT_PER_WAVE;
  const int Kc = a.k1 + a.k2;
  const int nkt = (Kc + 31) / 32;
  const int ntl = max(0, min(KT_PER_WAVE, nkt - kt0));
  const int64_t mbeg = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t mend = min(a.M, mbeg + a.rows_per_block);

  floatx16 acc[KT_PER_WAVE];
#pragma unroll
  for (int t = 0; t < KT_PER_WAVE; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  const int pn = tid & 127;  // prologue: column pn, rows rg*GR .. rg*GR+GR-1
  const int rg = tid >> 7;
  const bool colok = pn < a.Nr;
  const int pnc = colok ? pn : 0;
  float db = 0.0f;
  float dw2[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  float dzs = 0.f;  // column pn's dz sum (pn < MAXPROJ only)
  __shared__ float Ps[MAXPROJ * 128];  // projection columns (kept in LDS: saves 4 VGPRs per thread)
  if constexpr (PROJ) {
    if (tid < 128) {
#pragma unroll
      for (int q = 0; q < MAXPROJ; ++q) Ps[q * 128 + tid] = (q < a.nproj && tid < a.Nr) ? a.proj[q * a.Nr + tid] : 0.0f;
    }
    __syncthreads();  // Ps is read by every thread's first store_chunk
  }
  constexpr int NRG = TN_THREADS / 128;              // prologue row groups
  constexpr int GR = MC / NRG;                       // prologue rows per thread
  // A staging: 32 threads per chunk row; thread owns columns (tl*AVEC + 32*AVEC*j), j < AJ
  constexpr int TPR = TN_THREADS / MC;               // threads per row (32)
  constexpr int AJ = KMAX / (TPR * AVEC);            // vectors per thread per row
  const int ar = tid / TPR;                          // this thread's chunk row
  const int tl = tid - ar * TPR;
  float rg_in[GR][PROJ ? MAXPROJ : 1];
  float rh[GR];
  float ra[AJ][AVEC];

  auto load_chunk = [&](int64_t m0) {
#pragma unroll
    for (int i = 0; i < GR; ++i) {
      int64_t m = m0 + rg * GR + i;
      m = m < mend ? m : mend - 1;  // clamped: always a valid row, masked in store_chunk
      if constexpr (PROJ) {
        if (a.nproj == 4 && (a.lddz & 3) == 0) {
          float4 t = *reinterpret_cast<const float4*>(a.dz + m * a.lddz);
          rg_in[i][0] = t.x; rg_in[i][1] = t.y; rg_in[i][2] = t.z; rg_in[i][3] = t.w;
        } else {
#pragma unroll
          for (int q = 0; q < MAXPROJ; ++q) rg_in[i][q] = a.dz[m * a.lddz + (q < a.nproj ? q : 0)];
        }
      } else {
        rg_in[i][0] = a.g[m * a.ldg + pnc];
      }
      if constexpr (MASK) rh[i] = a.h[m * a.ldh + pnc];
    }
    int64_t m = m0 + ar;
    m = m < mend ? m : mend - 1;
    const float* b1 = a.a1 + m * a.lda1;
    const float* b2 = a.a2 + m * a.lda2 - a.k1;
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int k = tl * AVEC + TPR * AVEC * j;
      const float* src = k < a.k1 ? b1 + k : (k < Kc ? b2 + k : b1);
      if constexpr (AVEC == 2) {
        float2 t = *reinterpret_cast<const float2*>(src);
        ra[j][0] = t.x; ra[j][1] = t.y;
      } else {
        ra[j][0] = *src;
      }
    }
  };

  auto store_chunk = [&](int64_t m0, int buf) {
#pragma unroll
    for (int i = 0; i < GR; ++i) {
      const int r = rg * GR + i;
      const bool rok = m0 + r < mend;
      const bool ok = rok && colok;
      float g;
      if constexpr (PROJ) {
        g = rg_in[i][0] * Ps[pn];
#pragma unroll
        for (int q = 1; q < MAXPROJ; ++q) g = fmaf(rg_in[i][q], Ps[q * 128 + pn], g);
      } else {
        g = rg_in[i][0];
      }
      if constexpr (MASK) {
        g = rh[i] > 0.0f ? g * a.hscale : 0.0f;
        if constexpr (PROJ) {
#pragma unroll
          for (int q = 0; q < MAXPROJ; ++q) dw2[q] = fmaf(ok ? rg_in[i][q] : 0.0f, rh[i], dw2[q]);
        }
      }
      if constexpr (PROJ) {
        if (pn < MAXPROJ) dzs += rok ? rg_in[i][pn] : 0.0f;  // lanes 0..3 of each row group own one dz column
      }
      g = ok ? g : 0.0f;
      db += g;
      if (a.gout && ok) a.gout[(m0 + r) * a.ldgout + pn] = g;
      Gs[buf][r * 128 + pn] = g;
    }
    const bool rok = m0 + ar < mend;
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int k = tl * AVEC + TPR * AVEC * j;
      const bool ok = rok && k < Kc;
      if constexpr (AVEC == 2) {
        *reinterpret_cast<float2*>(&As[buf][ar * TN_APITCH + k]) = make_float2(ok ? ra[j][0] : 0.0f, ok ? ra[j][1] : 0.0f);
      } else {
        As[buf][ar * TN_APITCH + k] = ok ? ra[j][0] : 0.0f;
      }
    }
  };

  if (mbeg < mend) {
    load_chunk(mbeg);
    store_chunk(mbeg, 0);
    __syncthreads();
    int buf = 0;
    for (int64_t m0 = mbeg; m0 < mend; m0 += MC) {
      const bool more = m0 + MC < mend;
      if (more) load_chunk(m0 + MC);
      const float* gptr = Gs[buf] + (lane >> 5) * 128 + ntile * 32 + (lane & 31);
      const float* aptr = As[buf] + (lane >> 5) * TN_APITCH + (lane & 31);
      switch (ntl) {
        case 3: tn_mma<MC, 3>(acc, gptr, aptr, kt0); break;
        case 2: tn_mma<MC, 2>(acc, gptr, aptr, kt0); break;
        case 1: tn_mma<MC, 1>(acc, gptr, aptr, kt0); break;
        default: break;
      }
      if (more) store_chunk(m0 + MC, buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // ---- write this block's partial dW
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int t = 0; t < KT_PER_WAVE; ++t) {
    const int kt = kt0 + t;
    if (kt >= nkt) continue;
    const int col = kt * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = ntile * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      // segment-major: dW1 = [Nr][k1] then dW2 = [Nr][k2], each contiguous
      const int64_t idx = col < a.k1 ? (int64_t)row * a.k1 + col
                                     : (int64_t)a.Nr * a.k1 + (int64_t)row * a.k2 + (col - a.k1);
      if (row < a.Nr && col < Kc) slab[idx] = acc[t][r];
    }
  }
  // ---- side sums: reduce the 4 row groups through LDS (fixed order); reuse Gs as scratch
  float* red = &As[0][0];  // 2*MC*KMAX >= NRG*128*(1+MAXPROJ) floats for MC >= 16
  static_assert(2 * MC * TN_APITCH >= (TN_THREADS / 128) * 128 * (1 + MAXPROJ), "side-sum scratch");
  constexpr int ns = 1 + MAXPROJ;
  __syncthreads();
  red[(rg * 128 + pn) * ns + 0] = db;
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) red[(rg * 128 + pn) * ns + 1 + q] = dw2[q];
  __syncthreads();
  if (tid < 128 && colok) {
    float* side = slab + (int64_t)a.Nr * Kc;
    float s2 = 0.f;
    for (int g2 = 0; g2 < NRG; ++g2) s2 += red[(g2 * 128 + pn) * ns];
    side[pn] = s2;
    for (int q = 0; q < a.nproj; ++q) {
      float w = 0.f;
      for (int g2 = 0; g2 < NRG; ++g2) w += red[(g2 * 128 + pn) * ns + 1 + q];
      side[a.Nr + q * a.Nr + pn] = w;
    }
  }
  __syncthreads();
  if (pn < MAXPROJ) red[rg * MAXPROJ + pn] = dzs;
  __syncthreads();
  if (tid < a.nproj) {
    float s2 = 0.f;
    for (int g2 = 0; g2 < NRG; ++g2) s2 += red[g2 * MAXPROJ + tid];
    slab[(int64_t)a.Nr * Kc + a.Nr + a.nproj * a.Nr + tid] = s2;
  }
}

// out[j] = Σ_b slab[b][j], deterministic.  A 256-thread block owns 16 float4 outputs; its 16
// thread rows each sum a fixed 1/16 of the slabs (4 independent loads in flight), and the 16
// partials are combined through LDS in slab order.  ~700 blocks: the whole chip streams the
// slabs instead of one thread per output walking all of them.
// SqOut (ABI 20): the clip + Adam norm partials of this block's outputs (Σ out² and the count of
// non-finite outputs, outside [skip_lo, skip_hi)), and block 0 snapshots the optimizer's step count.
struct SqOut {
  float* part; const float* step; int64_t skip_lo, skip_hi;
};
constexpr int kRedOut = 16, kRedGrp = 16;
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab, int64_t stride, int nblk,
                                                          float* __restrict__ out, int64_t n, SqOut sq = SqOut{}) {
  __shared__ float4 part[kRedGrp][kRedOut];
  const int o = threadIdx.x & (kRedOut - 1);
  const int g = threadIdx.x / kRedOut;
  const int64_t j = ((int64_t)blockIdx.x * kRedOut + o) * 4;
  const int per = (nblk + kRedGrp - 1) / kRedGrp;
  const int b0 = g * per, b1 = min(nblk, b0 + per);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < n) {
    int b = b0;
    for (; b + 4 <= b1; b += 4) {
      float4 v0 = *reinterpret_cast<const float4*>(slab + (int64_t)(b + 0) * stride + j);
      float4 v1 = *reinterpret_cast<const float4*>(slab + (int64_t)(b + 1) * stride + j);
      float4 v2 = *reinterpret_cast<const float4*>(slab + (int64_t)(b + 2) * stride + j);
      float4 v3 = *reinterpret_cast<const float4*>(slab + (int64_t)(b + 3) * stride + j);
      s.x = (((s.x + v0.x) + v1.x) + v2.x) + v3.x;
      s.y = (((s.y + v0.y) + v1.y) + v2.y) + v3.y;
      s.z = (((s.z + v0.z) + v1.z) + v2.z) + v3.z;
      s.w = (((s.w + v0.w) + v1.w) + v2.w) + v3.w;
    }
    for (; b < b1; ++b) {
      float4 v = *reinterpret_cast<const float4*>(slab + (int64_t)b * stride + j);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  part[g][o] = s;
  __syncthreads();
  if (g != 0) return;  // threads 0..15 (wave 0) finish the block's 16 float4 outputs
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < n) {
    t = part[0][o];
    for (int q = 1; q < kRedGrp; ++q) {
      float4 v = part[q][o];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    if (j + 0 < n) out[j + 0] = t.x;
    if (j + 1 < n) out[j + 1] = t.y;
    if (j + 2 < n) out[j + 2] = t.z;
    if (j + 3 < n) out[j + 3] = t.w;
  }
  if (sq.part) {  // this block's norm partials: its 64 outputs in a fixed order (ABI 20)
    float s2 = 0.f, nf = 0.f;
    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t je = j + e;
      const bool use = je < n && (je < sq.skip_lo || je >= sq.skip_hi);
      s2 = use ? fmaf(tv[e], tv[e], s2) : s2;
      nf += (use && !isfinite(tv[e])) ? 1.f : 0.f;
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) {
      s2 += __shfl_xor(s2, off, 16);
      nf += __shfl_xor(nf, off, 16);
    }
    if (o == 0) {
      sq.part[blockIdx.x] = s2;
      sq.part[gridDim.x + blockIdx.x] = nf;
      if (blockIdx.x == 0) sq.part[2 * gridDim.x] = sq.step[0];
    }
  }
}

// Blocks of the TN launches: at most 256 (one per CU), and no more than the 32-row chunks need at
// the chunks-per-block that 256 blocks would take — every block has rows, so no block writes an
// all-zero slab for the reduce to read back (a strong-scaling shard: 213 instead of 256 slabs at
// 27,196 rows, -17 % of the slab traffic).
int tn_blocks(int64_t M) {
  const int64_t chunks = ceil_div(M, 32);
  if (chunks <= 0) return 1;
  const int64_t per = ceil_div(chunks, 256);
  return (int)ceil_div(chunks, per);
}
// the largest M whose half-pair dz-form TN runs split-K block pairs (GNNMP_TN_KSPLIT_MAXM, A/B)
static int64_t tn_ksplit_max_m() {
  static const int64_t v = [] {
    const char* e = std::getenv("GNNMP_TN_KSPLIT_MAXM");
    return e ? std::atoll(e) : (int64_t)32768;  // the 8-way shard (27k rows): TN + reduce 32.1 -> 30.9 us; 4-way (52k): slower
  }();
  return v;
}

// (ABI 26) the CSC sum of u inside the half-pair dz-form TN when each of its 8 waves walks at most
// one 64-row group of the block's rows (shard-sized M: 8-way shard 0.0947 -> 0.0923 ms per step,
// profiles/r105_csc_ab.txt); GNNMP_TN_CSC_INKERNEL=0 / 1 forces it off / on (A/B)
// rows per block of the half-pair TN (dz: the dz form, split-K pairs at shard-sized M)
static int64_t tn_h2_rows_per_block(int64_t M, bool dz) {
  const int64_t chunks = ceil_div(M, 32);
  if (dz && M <= tn_ksplit_max_m()) return ceil_div(chunks, 128) * 32;
  return ceil_div(chunks, tn_blocks(M)) * 32;
}
static bool tn_csc_in_kernel(int64_t rows_per_block) {
  static const int v = [] {
    const char* e = std::getenv("GNNMP_TN_CSC_INKERNEL");
    return e ? std::atoi(e) : -1;
  }();
  if (rows_per_block > 1792) return false;  // the block's dz rows staged in LDS (gemm_planes.hip dzb)
  if (v >= 0) return v != 0;
  return (rows_per_block + 63) / 64 + 1 <= 8;  // groups a block's rows can touch <= its waves
}

// the in-kernel half-pair TN at Nr <= 64, k1 + k2 <= 128 holds three blocks per CU (its LDS is
// sized by its k-tiles and 64 G rows, 47 KB): three times the blocks, so three times the chunk loads
// in flight per CU (its chunk loop is latency-bound: one 16-row chunk in flight per block)
int tn_blocks2(int64_t M) {
  const int64_t chunks = ceil_div(M, 32);
  if (chunks <= 0) return 1;
  const int64_t per = ceil_div(chunks, 768);
  return (int)ceil_div(chunks, per);
}

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

static gnn_status gemm_nt_dispatch(const gnn_gemm_nt_params* p, gnn_stream_t stream, const char* fn, int phase) {
  if (!p) return fail(GNN_ERR_INVALID_ARG, fn, "null params");
  if (phase == NT_PHASE_ALL && p->b_ready) phase = NT_PHASE_RUN;
  const bool planes_only = p->a_planes && !p->a1;  // A given only as a split image
  if (p->M < 0 || p->N < 1 || p->k1 < 1 || p->k2 < 0 || (!p->a1 && !p->a_planes) ||
      (p->k2 > 0 && !p->a2 && !planes_only))
    return fail(GNN_ERR_INVALID_ARG, fn, "bad shapes / null operands");
  if (!p->bt && !(p->w1 && (p->k2 == 0 || p->w2)))
    return fail(GNN_ERR_INVALID_ARG, fn, "need bt or w1 (and w2 when k2 > 0)");
  if (p->w1 && (p->N > BN || p->ldw1 < p->k1 || (p->k2 > 0 && p->ldw2 < p->k2)))
    return fail(GNN_ERR_INVALID_ARG, fn, "w1/w2 form needs N <= 128 and ldw >= k");
  if ((!planes_only && (p->lda1 < p->k1 || (p->k2 > 0 && p->lda2 < p->k2))) || (p->bt && p->ldb < p->N) ||
      (p->c && p->ldc < p->N))
    return fail(GNN_ERR_INVALID_ARG, fn, "bad leading dimensions");
  if (p->nproj < 0 || p->nproj > 4 || (p->nproj > 0 && (p->N > BN || !p->proj || !p->z || p->ldz < p->nproj)))
    return fail(GNN_ERR_INVALID_ARG, fn, "projection needs N <= 128, nproj <= 4, proj and z");
  if (p->dropout_p < 0.f || p->dropout_p >= 1.f) return fail(GNN_ERR_INVALID_ARG, fn, "dropout p in [0,1)");
  if (p->dropout_p > 0.f && (int64_t)p->M * (int64_t)p->N >= ((int64_t)1 << 32))
    return fail(GNN_ERR_UNSUPPORTED, fn, "dropout element index (rows x width) must be < 2^32");
  if (p->math != GNN_MATH_SPLIT_BF16 && p->math != GNN_MATH_F32 && p->math != GNN_MATH_HALF_PAIR)
    return fail(GNN_ERR_INVALID_ARG, fn, "bad math mode");
  if ((p->a_dtype != GNN_DTYPE_F32 && p->a_dtype != GNN_DTYPE_BF16) || (p->c_dtype != GNN_DTYPE_F32 && p->c_dtype != GNN_DTYPE_BF16))
    return fail(GNN_ERR_INVALID_ARG, fn, "bad dtype");
  if (p->row_exp && (p->a_planes || p->colsum_part || phase != NT_PHASE_ALL))
    return fail(GNN_ERR_UNSUPPORTED, fn, "row_exp needs the in-kernel half-pair NT over f32 A1 / A2");
  if (p->M == 0 && phase != NT_PHASE_PREP) return GNN_OK;
  NTArgs a{};
  a.M = p->M; a.Nc = (int32_t)p->N;
  a.a1 = p->a1; a.lda1 = p->lda1; a.k1 = (int32_t)p->k1;
  a.a2 = p->a2; a.lda2 = p->lda2; a.k2 = (int32_t)p->k2;
  a.bt = p->bt; a.ldb = p->ldb; a.w1 = p->w1; a.w2 = p->w2; a.ldw1 = p->ldw1; a.ldw2 = p->ldw2; a.c = p->c;
  a.ldc = p->ldc; a.bias = p->bias; a.relu = p->relu;
  a.dropout = p->dropout_p > 0.f;
  a.keep_thresh = (uint32_t)((1.0 - (double)p->dropout_p) * 16777216.0);
  a.drop_scale = a.dropout ? (float)(1.0 / (1.0 - (double)p->dropout_p)) : 1.0f;
  a.seed = p->seed;
  a.seed_ptr = p->seed_ptr;
  a.proj = p->proj; a.nproj = p->nproj; a.z = p->z; a.ldz = p->ldz;
  auto al = [](const void* q, int b) { return (reinterpret_cast<uintptr_t>(q) % b) == 0; };
  a.wvec2 = a.w1 && (a.ldw1 % 2 == 0) && (a.k1 % 2 == 0) && al(a.w1, 8) &&
            (a.k2 == 0 || ((a.ldw2 % 2 == 0) && (a.k2 % 2 == 0) && al(a.w2, 8)));
  auto wv = [&](int v) {
    return a.w1 && (a.ldw1 % v == 0) && (a.k1 % v == 0) && al(a.w1, 4 * v) &&
           (a.k2 == 0 || ((a.ldw2 % v == 0) && (a.k2 % v == 0) && al(a.w2, 4 * v)));
  };
  a.wvec = wv(4) ? 4 : (wv(2) ? 2 : 1);
  bool v4 = (a.k1 % 4 == 0) && (a.lda1 % 4 == 0) && al(a.a1, 16) &&
            (a.k2 == 0 || ((a.k2 % 4 == 0) && (a.lda2 % 4 == 0) && al(a.a2, 16)));
  bool v2 = (a.k1 % 2 == 0) && (a.lda1 % 2 == 0) && al(a.a1, 8) &&
            (a.k2 == 0 || ((a.k2 % 2 == 0) && (a.lda2 % 2 == 0) && al(a.a2, 8)));
  hipStream_t st = (hipStream_t)stream;
  a.a_bf16 = p->a_dtype == GNN_DTYPE_BF16;
  a.c_bf16 = p->c_dtype == GNN_DTYPE_BF16;
  a.mask = p->mask; a.ldmask = p->ldmask; a.mask_scale = p->mask_scale;
  if (p->mask && p->ldmask < p->N) return fail(GNN_ERR_INVALID_ARG, fn, "bad ldmask");
  if (p->colsum_part) {  // ABI 21: the skinny-K form also writes C's per-block column sums
    const int nb = nt_skinny_k_blocks(a);
    if (nb == 0 || p->a_planes || phase != NT_PHASE_ALL)
      return fail(GNN_ERR_UNSUPPORTED, fn, "colsum_part needs the skinny-K form (k1 <= 8, k2 = 0, 8 < N <= 256)");
    if (p->colsum_cap < (int64_t)nb * p->N || (reinterpret_cast<uintptr_t>(p->colsum_part) & 3))
      return fail(GNN_ERR_INVALID_ARG, fn, "colsum_cap < gnn_gemm_nt_colsum_blocks x N");
    a.colsum_part = p->colsum_part;
    if (!launch_nt_skinny(a, st)) return fail(GNN_ERR_UNSUPPORTED, fn, "colsum_part: not the skinny-K form");
    return hip_check(hipGetLastError(), fn);
  }
  if (p->a_planes) {
    if (p->planes_format != GNN_PLANES_SPLIT_BF16 && p->planes_format != GNN_PLANES_HALF_PAIR)
      return fail(GNN_ERR_INVALID_ARG, fn, "bad planes_format");
    a.ap = static_cast<const uint16_t*>(p->a_planes);
    a.ap_ld = (int32_t)std::min<int64_t>(p->planes_ld, INT32_MAX);
    a.ap_col2 = (int32_t)std::min<int64_t>(p->planes_col2, INT32_MAX);
    a.ap_ps = p->planes_stride;
    a.ap_h2 = p->planes_format == GNN_PLANES_HALF_PAIR;
    a.ap_exp = a.ap_h2 ? p->planes_exp : 0;
    if (a.ap_exp < -100 || a.ap_exp > 100) return fail(GNN_ERR_INVALID_ARG, fn, "planes_exp outside [-100, 100]");
    const size_t img_bytes = (size_t)(a.ap_ld / 16) * 3 * 256 * sizeof(uint4);
    if (p->keep_mask) {
      if (!a.ap_h2 || !a.dropout || (reinterpret_cast<uintptr_t>(p->keep_mask) & 3))
        return fail(GNN_ERR_INVALID_ARG, fn, "keep_mask needs a half-pair image A and dropout_p > 0");
      a.kmask = p->keep_mask;
    }
    if (a.ap_h2) {  // the half-pair image: f16 hi / lo planes, 3 products
      if (p->math != GNN_MATH_F32 && !p->mask && nt_h2_ok(a) && p->workspace &&
          p->workspace_bytes >= img_bytes + BN * sizeof(float)) {
        launch_nt_h2(a, static_cast<uint4*>(p->workspace), st, phase);
        return hip_check(hipGetLastError(), fn);
      }
      if (planes_only) return fail(GNN_ERR_UNSUPPORTED, fn, "half-pair image A outside the half-pair kernel's shapes");
      a.ap = nullptr;
    }
    if (a.a_bf16) {  // a bf16 image (one plane): the bf16-storage form
      if (p->math != GNN_MATH_F32 && !p->mask && nt_img16_ok(a) && p->workspace && p->workspace_bytes >= img_bytes) {
        launch_nt_img16(a, static_cast<uint4*>(p->workspace), st, phase);
        return hip_check(hipGetLastError(), fn);
      }
      return fail(GNN_ERR_UNSUPPORTED, fn, "bf16 image A outside the image kernel's shapes");
    }
    if (p->math != GNN_MATH_F32 && !p->mask && nt_planes_ok(a) && p->workspace &&
        p->workspace_bytes >= img_bytes) {
      launch_nt_ws_planes(a, static_cast<uint4*>(p->workspace), st, phase);
      return hip_check(hipGetLastError(), fn);
    }
    if (planes_only) return fail(GNN_ERR_UNSUPPORTED, fn, "split-image A outside the planes kernel's shapes");
    a.ap = nullptr;  // the f32 operands serve
  }
  if (phase != NT_PHASE_ALL)  // prep_b / b_ready: only the image-A kernels have a separate B image
    return fail(phase == NT_PHASE_PREP ? GNN_ERR_UNSUPPORTED : GNN_ERR_INVALID_ARG, fn,
                "a separate B prep (prep_b / b_ready) needs an image-A kernel (gnn_gemm_nt_planes_ok)");
  const bool h2s = p->math == GNN_MATH_HALF_PAIR && nt_h2s_ok(a) && p->workspace &&
                   p->workspace_bytes >= nt_h2s_workspace(a.k1, a.k2);
  if (p->row_exp && !h2s)  // (checked before the skinny forms: a caller asking for row_exp gets it or an error)
    return fail(GNN_ERR_UNSUPPORTED, fn, "row_exp needs the in-kernel half-pair NT (GNN_MATH_HALF_PAIR, the w1/w2 "
                                         "form, N <= 128, k1 / k2 multiples of 16, k1 + k2 <= 128, f32, a workspace)");
  if (!p->row_exp && launch_nt_skinny(a, st)) return hip_check(hipGetLastError(), fn);  // Nc <= 8 or K <= 8
  if (p->mask) return fail(GNN_ERR_UNSUPPORTED, fn, "the mask epilogue needs a skinny shape (K <= 8 or N <= 8)");
  if (a.a_bf16 || a.c_bf16) {
    if (!a.a_bf16 || !a.w1 || a.Nc > BN || p->math == GNN_MATH_F32)
      return fail(GNN_ERR_UNSUPPORTED, fn, "bf16 NT needs bf16 A, the w1/w2 form, N <= 128 and split math");
    launch_nt_x3(a, p->workspace, p->workspace_bytes, st);
    return hip_check(hipGetLastError(), fn);
  }
  if (h2s) {  // in-kernel half-pair (gemm_x3.hip, ABI 23)
    a.rowexp = p->row_exp;
    launch_nt_h2s(a, p->workspace, st);
    return hip_check(hipGetLastError(), fn);
  }
  if (p->math != GNN_MATH_F32 && a.w1 && a.Nc <= BN) {
    launch_nt_x3(a, p->workspace, p->workspace_bytes, st);  // split-bf16 MFMA (gemm_x3.hip)
    return hip_check(hipGetLastError(), fn);
  }
  if (v4) launch_nt_f32<4>(a, st);
  else if (v2) launch_nt_f32<2>(a, st);
  else launch_nt_f32<1>(a, st);
  return hip_check(hipGetLastError(), fn);
}

extern "C" gnn_status gnn_gemm_nt_workspace_size(int64_t N, int64_t k1, int64_t k2, size_t* bytes) {
  if (!bytes || N < 1 || k1 < 1 || k2 < 0) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  // the image-A kernels (a_planes) size their B image by the image's row width (<= 336 columns,
  // 21 k-steps), not by k1 + k2: a narrow input on a 176-wide image runs 11 k-steps
  *bytes = N <= BN ? std::max(nt_x3_workspace(k1, k2), (size_t)21 * 3 * 256 * 16 + BN * sizeof(float)) : 0;
  return GNN_OK;
}

extern "C" gnn_status gnn_gemm_nt_f32(const gnn_gemm_nt_params* p, gnn_stream_t stream) {
  return gemm_nt_dispatch(p, stream, __func__, NT_PHASE_ALL);
}

extern "C" gnn_status gnn_gemm_nt_prep_b(const gnn_gemm_nt_params* p, gnn_stream_t stream) {
  return gemm_nt_dispatch(p, stream, __func__, NT_PHASE_PREP);
}


extern "C" gnn_status gnn_gemm_tn_workspace_size(int64_t M, int64_t Nr, int64_t Kc, int32_t nproj, size_t* bytes) {
  if (!bytes || M < 0 || Nr < 1 || Kc < 1 || nproj < 0) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  int64_t stride = Nr * Kc + Nr + (int64_t)nproj * Nr + nproj;
  stride = (stride + 63) / 64 * 64;
  int64_t nb = tn_blocks(M);
  if (Nr <= 8 && nproj == 0) nb = std::max<int64_t>(nb, tn_skinny_blocks(M));  // gemm_skinny.hip
  if (Nr <= 64 && Kc <= 128 && nproj == 0) nb = std::max<int64_t>(nb, tn_blocks2(M));  // the narrow half-pair TN
  *bytes = (size_t)nb * stride * sizeof(float);
  return GNN_OK;
}

static gnn_status gemm_tn_dispatch(const gnn_gemm_tn_params* p, float* out, void* workspace,
                                   size_t workspace_bytes, gnn_stream_t stream);

// (ABI 26) the folded CSC sum's arguments (dz_graph's CSC, dz_u, dz_cols); false when dz_graph is
// given but cannot be taken (no dz form, no u, dz_cols outside 1..min(2, nproj), num_nodes != M)
static bool tn_csc_args(const gnn_gemm_tn_params* p, TNArgs* a) {
  a->cptr = nullptr; a->cnbr = nullptr; a->cu = nullptr; a->ldu = 0; a->ccols = 0;
  const gnn_graph* cg = p->dz_graph;
  if (!cg) return true;
  if (!p->dz || !p->dz_u || !cg->colptr || !cg->row || cg->num_nodes != p->M || p->dz_cols < 1 || p->dz_cols > 2 ||
      p->dz_cols > p->nproj || p->ldu < p->dz_cols)
    return false;
  a->cptr = cg->colptr; a->cnbr = cg->row; a->cu = p->dz_u; a->ldu = p->ldu; a->ccols = p->dz_cols;
  return true;
}

static unsigned red_blocks(int64_t n_out) { return (unsigned)ceil_div(ceil_div(n_out, 4), kRedOut); }

extern "C" gnn_status gnn_gemm_tn_sq_blocks(int64_t n_out, int32_t* nb) {
  if (!nb || n_out < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  *nb = (int32_t)red_blocks(n_out);
  return GNN_OK;
}

extern "C" gnn_status gnn_gemm_tn_f32(const gnn_gemm_tn_params* p, float* out, void* workspace,
                                      size_t workspace_bytes, gnn_stream_t stream) {
  return gemm_tn_dispatch(p, out, workspace, workspace_bytes, stream);
}


static gnn_status gemm_tn_dispatch(const gnn_gemm_tn_params* p, float* out, void* workspace,
                                   size_t workspace_bytes, gnn_stream_t stream) {
  const char* __fn = "gnn_gemm_tn_f32";
  if (!p || !out) return fail(GNN_ERR_INVALID_ARG, __fn, "null params/out");
  if (p->M < 0 || p->Nr < 1 || p->Nr > 128 || p->k1 < 1 || p->k2 < 0 || p->k1 + p->k2 > KMAX)
    return fail(GNN_ERR_UNSUPPORTED, __fn, "needs 1 <= Nr <= 128 and k1 + k2 <= 384");
  const bool planes_only = p->a_planes && !p->a1;
  if (!planes_only && (!p->a1 || (p->k2 > 0 && !p->a2) || p->lda1 < p->k1 || (p->k2 > 0 && p->lda2 < p->k2)))
    return fail(GNN_ERR_INVALID_ARG, __fn, "bad A operands");
  if (p->dz) {
    if (p->nproj < 1 || p->nproj > MAXPROJ || !p->proj || p->lddz < p->nproj)
      return fail(GNN_ERR_INVALID_ARG, __fn, "dz form needs 1 <= nproj <= 4 and proj");
  } else if (!p->g || p->ldg < p->Nr) {
    return fail(GNN_ERR_INVALID_ARG, __fn, "need g (or dz + proj)");
  }
  if (p->h && p->ldh < p->Nr) return fail(GNN_ERR_INVALID_ARG, __fn, "bad ldh");
  if (p->math != GNN_MATH_SPLIT_BF16 && p->math != GNN_MATH_F32 && p->math != GNN_MATH_HALF_PAIR)
    return fail(GNN_ERR_INVALID_ARG, __fn, "bad math mode");
  if (p->gout && p->ldgout < p->Nr) return fail(GNN_ERR_INVALID_ARG, __fn, "bad ldgout");
  const int32_t nproj = p->dz ? p->nproj : 0;
  const int64_t Kc = p->k1 + p->k2;
  const int64_t n_out = p->Nr * Kc + p->Nr + (int64_t)nproj * p->Nr + nproj;
  int64_t stride = (n_out + 63) / 64 * 64;
  int nblk = tn_blocks(p->M);
  if (!workspace || workspace_bytes < (size_t)nblk * stride * sizeof(float))
    return fail(GNN_ERR_WORKSPACE, __fn, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  SqOut sqo{};
  if (p->sq_partial) {
    if (!p->sq_step || p->sq_cap < 2 * (int64_t)red_blocks(n_out) + 1 || p->sq_skip_lo > p->sq_skip_hi)
      return fail(GNN_ERR_INVALID_ARG, __fn, "sq_partial needs sq_step, sq_cap >= 2 nb + 1, skip_lo <= skip_hi");
    sqo = SqOut{p->sq_partial, p->sq_step, p->sq_skip_lo, p->sq_skip_hi};
  }
  if (p->M == 0) {
    if (!p->sq_partial) return hip_check(hipMemsetAsync(out, 0, n_out * sizeof(float), st), __fn);
    slab_reduce_kernel<<<red_blocks(n_out), 256, 0, st>>>(static_cast<float*>(workspace), stride, 0, out, n_out, sqo);
    return hip_check(hipGetLastError(), __fn);  // zero slabs: out = 0, partials 0, the step snapshot
  }
  TNArgs a{};
  a.M = p->M; a.Nr = (int32_t)p->Nr;
  a.g = p->g; a.ldg = p->ldg; a.dz = p->dz; a.lddz = p->lddz; a.proj = p->proj; a.nproj = nproj;
  a.h = p->h; a.ldh = p->ldh; a.hscale = p->hscale;
  a.gout = p->gout; a.ldgout = p->ldgout;
  a.a1 = p->a1; a.lda1 = p->lda1; a.k1 = (int32_t)p->k1;
  a.a2 = p->a2; a.lda2 = p->lda2; a.k2 = (int32_t)p->k2;
  a.slab = static_cast<float*>(workspace); a.slab_stride = stride;
  a.rows_per_block = ceil_div(ceil_div(p->M, 32), nblk) * 32;  // multiple of both chunk sizes
  if (!tn_csc_args(p, &a))
    return fail(GNN_ERR_INVALID_ARG, __fn, "dz_graph needs the dz form, dz_u, 1 <= dz_cols <= 2 and num_nodes == M");
  auto al8 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 7) == 0; };
  const bool v2 = (a.k1 % 2 == 0) && (a.lda1 % 2 == 0) && al8(a.a1) &&
                  (a.k2 == 0 || ((a.k2 % 2 == 0) && (a.lda2 % 2 == 0) && al8(a.a2)));
  const bool proj = a.dz != nullptr, mask = a.h != nullptr;
  a.a_bf16 = p->a_dtype == GNN_DTYPE_BF16;
  a.h_bf16 = p->h_dtype == GNN_DTYPE_BF16;
  a.g_bf16 = p->g_dtype == GNN_DTYPE_BF16;
  if ((p->a_dtype != GNN_DTYPE_F32 && p->a_dtype != GNN_DTYPE_BF16) || (p->h_dtype != GNN_DTYPE_F32 && p->h_dtype != GNN_DTYPE_BF16) ||
      (p->g_dtype != GNN_DTYPE_F32 && p->g_dtype != GNN_DTYPE_BF16))
    return fail(GNN_ERR_INVALID_ARG, __fn, "bad dtype");
  if (a.g_bf16 && !(p->a_planes && a.a_bf16))
    return fail(GNN_ERR_UNSUPPORTED, __fn, "bf16 g / gout need the bf16-image TN (a bf16 a_planes)");
  if (a.h_bf16 && !a.a_bf16) return fail(GNN_ERR_UNSUPPORTED, __fn, "bf16 h needs bf16 A");
  // widest row pitch of any operand (the split kernel uses 32-bit element offsets)
  const int64_t ldmax = std::max({a.lda1, a.k2 > 0 ? a.lda2 : 0, a.h ? a.ldh : 0, a.g ? a.ldg : 0, a.dz ? a.lddz : 0});
  if (p->a_planes) {
    if (p->planes_format != GNN_PLANES_SPLIT_BF16 && p->planes_format != GNN_PLANES_HALF_PAIR)
      return fail(GNN_ERR_INVALID_ARG, __fn, "bad planes_format");
    a.ap = static_cast<const uint16_t*>(p->a_planes);
    a.ap_ld = (int32_t)std::min<int64_t>(p->planes_ld, INT32_MAX);
    a.ap_col2 = (int32_t)std::min<int64_t>(p->planes_col2, INT32_MAX);
    a.ap_ps = p->planes_stride;
    a.ap_h2 = p->planes_format == GNN_PLANES_HALF_PAIR;
    a.ap_exp = a.ap_h2 ? p->planes_exp : 0;
    if (a.ap_exp < -100 || a.ap_exp > 100) return fail(GNN_ERR_INVALID_ARG, __fn, "planes_exp outside [-100, 100]");
    if (a.ap_h2) {  // the half-pair image: f16 hi / lo planes, 3 products
      // (ABI 25) the plain g form's block scale from the producer's row-group maxima (row blocks are
      // whole 32-row chunks, so every block covers whole GNN_ROWMAX_ROWS groups)
      a.growmax = (!a.dz && a.g) ? p->g_rowmax : nullptr;
      if (p->math != GNN_MATH_F32 && tn_h2_ok(a)) {
        // a shard-sized M (the dz form): split-K block pairs over half as many row blocks (round 6)
        int nred = nblk;
        const bool ks = a.dz && a.M <= tn_ksplit_max_m();
        if (ks) {
          const int64_t chunks = ceil_div(a.M, 32), per = ceil_div(chunks, 128);
          nred = (int)ceil_div(chunks, per);
          a.rows_per_block = per * 32;
        }
        if (a.rows_per_block != tn_h2_rows_per_block(a.M, a.dz != nullptr))
          return fail(GNN_ERR_HIP, __fn, "internal: TN row-block rule mismatch");
        if (a.cptr && !tn_csc_in_kernel(a.rows_per_block)) {
          // (ABI 26) rows of more than one 64-row group per wave: the folded CSC sum would run two
          // dependent gather rounds per wave ahead of the chunk loop (full configs[1] graph, 800 rows a
          // block: TN 87 -> 94 us, profiles/r105_csc_ab.txt) — the separate narrow launch instead
          gnn_agg_params ag{};
          ag.mode = GNN_AGG_SUM;
          ag.transpose = 1;
          const gnn_status s = gnn_aggregate_f32(p->dz_graph, &ag, p->dz_u, p->ldu, p->dz_cols,
                                                 const_cast<float*>(p->dz), p->lddz, stream);
          if (s != GNN_OK) return s;
          a.cptr = nullptr;
        }
        launch_tn_h2(a, ks ? 2 * nred : nblk, st, ks);
        GNN_LAUNCH_CHECK();
        slab_reduce_kernel<<<red_blocks(n_out), 256, 0, st>>>(a.slab, stride, nred, out, n_out, sqo);
        GNN_LAUNCH_CHECK();
        return GNN_OK;
      }
      if (planes_only) return fail(GNN_ERR_UNSUPPORTED, __fn, "half-pair image A outside the half-pair kernel's shapes");
      a.ap = nullptr;
    }
  }
  if (a.cptr)  // only the half-pair dz-form kernel forms dz's CSC columns itself
    return fail(GNN_ERR_UNSUPPORTED, __fn, "dz_graph outside the half-pair dz-form TN (gnn_gemm_tn_planes_ok)");
  if (p->a_planes) {
    if (a.ap && a.a_bf16) {  // a bf16 image (one plane): the bf16-storage form
      if (p->math == GNN_MATH_F32 || !tn_img16_ok(a))
        return fail(GNN_ERR_UNSUPPORTED, __fn, "bf16 image A outside the image kernel's shapes");
      launch_tn_img16(a, nblk, st);
      GNN_LAUNCH_CHECK();
      slab_reduce_kernel<<<red_blocks(n_out), 256, 0, st>>>(a.slab, stride, nblk, out, n_out, sqo);
      GNN_LAUNCH_CHECK();
      return GNN_OK;
    }
    if (a.ap && p->math != GNN_MATH_F32 && tn_planes_ok(a)) {
      launch_tn_planes(a, nblk, st);
      GNN_LAUNCH_CHECK();
      slab_reduce_kernel<<<red_blocks(n_out), 256, 0, st>>>(a.slab, stride, nblk, out, n_out, sqo);
      GNN_LAUNCH_CHECK();
      return GNN_OK;
    }
    if (planes_only) return fail(GNN_ERR_UNSUPPORTED, __fn, "split-image A outside the planes kernel's shapes");
    a.ap = nullptr;
  }
  if (tn_skinny_ok(a)) {  // Nr <= 8 plain g form: VALU stream (gemm_skinny.hip)
    nblk = tn_skinny_blocks(a.M);
    if (workspace_bytes < (size_t)nblk * stride * sizeof(float))
      return fail(GNN_ERR_WORKSPACE, __fn, "workspace too small");
    launch_tn_skinny(a, nblk, st);
    GNN_LAUNCH_CHECK();
    slab_reduce_kernel<<<red_blocks(n_out), 256, 0, st>>>(a.slab, stride, nblk, out, n_out, sqo);
    GNN_LAUNCH_CHECK();
    return GNN_OK;
  }
  // the split kernel indexes rows with 32-bit element offsets and loads whole 16-row chunks
  if (a.a_bf16 && (p->math == GNN_MATH_F32 || (a.M + 32) * ldmax >= ((int64_t)1 << 31) || a.M < 16))
    return fail(GNN_ERR_UNSUPPORTED, __fn, "bf16 TN needs split math, M >= 16 and M*ld < 2^31");
  a.rowexp = p->row_exp;
  if (p->math == GNN_MATH_HALF_PAIR && tn_h2s_ok(a) && (a.M + 32) * ldmax < ((int64_t)1 << 31)) {
    if (a.Nr <= 64 && Kc <= 128 && !nproj && workspace_bytes >= (size_t)tn_blocks2(a.M) * stride * sizeof(float)) {
      nblk = tn_blocks2(a.M);
      a.rows_per_block = ceil_div(ceil_div(a.M, 32), nblk) * 32;
    }
    launch_tn_h2s(a, nblk, st);  // in-kernel half-pair MFMA (gemm_x3.hip, ABI 23)
    GNN_LAUNCH_CHECK();
    slab_reduce_kernel<<<red_blocks(n_out), 256, 0, st>>>(a.slab, stride, nblk, out, n_out, sqo);
    GNN_LAUNCH_CHECK();
    return GNN_OK;
  }
  if (p->math != GNN_MATH_F32 && (a.M + 32) * ldmax < ((int64_t)1 << 31) && a.M >= 16) {
    launch_tn_x3(a, nblk, st);  // split-bf16 MFMA (gemm_x3.hip)
    GNN_LAUNCH_CHECK();
    slab_reduce_kernel<<<red_blocks(n_out), 256, 0, st>>>(a.slab, stride, nblk, out, n_out, sqo);
    GNN_LAUNCH_CHECK();
    return GNN_OK;
  }
#define GNN_TN(P, MK, V, R) gemm_tn_kernel<P, MK, V, R><<<nblk, TN_THREADS, 0, st>>>(a)
  // the dz·P + mask prologue holds twice the staging registers: 16-row chunks keep it spill-free
  if (proj && mask) { if (v2) GNN_TN(true, true, 2, 16); else GNN_TN(true, true, 1, 16); }
  else if (proj) { if (v2) GNN_TN(true, false, 2, 32); else GNN_TN(true, false, 1, 32); }
  else if (mask) { if (v2) GNN_TN(false, true, 2, 32); else GNN_TN(false, true, 1, 32); }
  else { if (v2) GNN_TN(false, false, 2, 32); else GNN_TN(false, false, 1, 32); }
#undef GNN_TN
  GNN_LAUNCH_CHECK();
  slab_reduce_kernel<<<red_blocks(n_out), 256, 0, st>>>(a.slab, stride, nblk, out, n_out, sqo);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

// Whether a call would run the split-image kernels (the caller then needs no f32 A).
static NTArgs nt_image_args(const gnn_gemm_nt_params* p) {  // the fields the image-A predicates read
  NTArgs a{};
  a.M = p->M; a.Nc = (int32_t)p->N; a.k1 = (int32_t)p->k1; a.k2 = (int32_t)p->k2;
  a.w1 = p->w1; a.w2 = p->w2; a.ldw1 = p->ldw1; a.ldw2 = p->ldw2;
  a.c = p->c; a.ldc = p->ldc; a.bias = p->bias; a.relu = p->relu;
  a.dropout = p->dropout_p > 0.f; a.nproj = p->nproj; a.ldz = p->ldz;
  a.a_bf16 = p->a_dtype == GNN_DTYPE_BF16; a.c_bf16 = p->c_dtype == GNN_DTYPE_BF16;
  a.ap = static_cast<const uint16_t*>(p->a_planes);
  a.ap_ld = (int32_t)std::min<int64_t>(p->planes_ld, INT32_MAX);
  a.ap_col2 = (int32_t)std::min<int64_t>(p->planes_col2, INT32_MAX);
  a.ap_ps = p->planes_stride;
  a.ap_h2 = p->planes_format == GNN_PLANES_HALF_PAIR;
  a.ap_exp = a.ap_h2 ? p->planes_exp : 0;
  return a;
}

extern "C" gnn_status gnn_gemm_nt_colsum_blocks(const gnn_gemm_nt_params* p, int32_t* nb) {
  if (!p || !nb) return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  NTArgs a = nt_image_args(p);
  *nb = p->a_planes ? 0 : nt_skinny_k_blocks(a);
  return GNN_OK;
}

extern "C" int gnn_gemm_nt_planes_ok(const gnn_gemm_nt_params* p) {
  if (!p || !p->a_planes || p->math == GNN_MATH_F32 || p->mask || p->M < 1) return 0;
  const NTArgs a = nt_image_args(p);
  if (a.ap_h2) return nt_h2_ok(a) ? 1 : 0;
  return (a.a_bf16 ? nt_img16_ok(a) : nt_planes_ok(a)) ? 1 : 0;
}

namespace gnnmp {
gnn_status nt_h2_prep_from_params(const gnn_gemm_nt_params* p, H2Prep* out, const char* fn) {
  if (!p || !p->a_planes || p->math == GNN_MATH_F32 || p->mask || p->M < 1 || p->planes_format != GNN_PLANES_HALF_PAIR)
    return fail(GNN_ERR_UNSUPPORTED, fn, "prep_b needs NT params that select the half-pair NT");
  const NTArgs a = nt_image_args(p);
  const size_t img_bytes = (size_t)(a.ap_ld / 16) * 3 * 256 * sizeof(uint4);
  if (a.ap_exp < -100 || a.ap_exp > 100) return fail(GNN_ERR_INVALID_ARG, fn, "planes_exp outside [-100, 100]");
  if (!nt_h2_ok(a) || !p->workspace || p->workspace_bytes < img_bytes + BN * sizeof(float) ||
      (reinterpret_cast<uintptr_t>(p->workspace) & 15))
    return fail(GNN_ERR_UNSUPPORTED, fn, "prep_b needs NT params that select the half-pair NT (and its workspace)");
  *out = h2_prep_of(a, static_cast<uint4*>(p->workspace));
  return GNN_OK;
}
}  // namespace gnnmp

extern "C" int gnn_gemm_tn_planes_ok(const gnn_gemm_tn_params* p) {
  if (!p || !p->a_planes || p->math == GNN_MATH_F32 || p->M < 1 || p->Nr < 1 || p->Nr > 128) return 0;
  TNArgs a{};
  a.M = p->M; a.Nr = (int32_t)p->Nr; a.g = p->g; a.ldg = p->ldg; a.dz = p->dz; a.lddz = p->lddz;
  a.h = p->h; a.ldh = p->ldh; a.gout = p->gout; a.ldgout = p->ldgout; a.k1 = (int32_t)p->k1; a.k2 = (int32_t)p->k2;
  a.a_bf16 = p->a_dtype == GNN_DTYPE_BF16; a.h_bf16 = p->h_dtype == GNN_DTYPE_BF16;
  a.g_bf16 = p->g_dtype == GNN_DTYPE_BF16;
  a.ap = static_cast<const uint16_t*>(p->a_planes);
  a.ap_ld = (int32_t)std::min<int64_t>(p->planes_ld, INT32_MAX);
  a.ap_col2 = (int32_t)std::min<int64_t>(p->planes_col2, INT32_MAX);
  a.ap_ps = p->planes_stride;
  a.ap_h2 = p->planes_format == GNN_PLANES_HALF_PAIR;
  if (!tn_csc_args(p, &a)) return 0;
  if (a.ap_h2) {
    a.proj = p->proj; a.nproj = p->dz ? p->nproj : 0;
    // (ABI 26) with dz_graph: 1 only when the kernel forms dz's CSC columns itself (a shard-sized
    // row block); the call would otherwise launch the CSC sum first, which the caller can as well
    if (a.cptr && !tn_csc_in_kernel(tn_h2_rows_per_block(a.M, true))) return 0;
    return tn_h2_ok(a) ? 1 : 0;
  }
  return (!a.cptr && (a.a_bf16 ? tn_img16_ok(a) : tn_planes_ok(a))) ? 1 : 0;
}
