// Split images ("planes") and the TN weight-gradient GEMM that reads them.
//
// The split-bf16 GEMMs (gemm_x3.hip, gemm_ws.hip) run every f32 operand as hi + mid + lo bf16
// terms.  Splitting an [N, K] operand costs ~5.5 VALU per element, and the layer-1 operand
// [agg | x] of the SAGE preset (N = 203,769, K = 332) is split twice per step (forward NT and
// backward TN) inside kernels whose MFMA phase should hide everything else: r08-r10 profiles put
// the split at ~265 of ~420 VALU per 16-row TN chunk and ~27 us of the NT.  A split image holds
// the three planes in HBM instead:
//
//   img[p][r][c]  (bf16; p = hi / mid / lo; row pitch ld; plane stride ps)
//   A1 (agg) in columns [0, k1), A2 (x) in [col2, col2 + k2), zeros elsewhere
//
// written by K1 (agg, every step: gnn_sage_mean_fwd_planes) and by gnn_split_planes_f32 (x,
// once per input tensor: x is a constant of the training run, like the CSR plan).  The GEMMs then
// stage A by plain 16-byte copies: 6 B per element instead of 4 B, no split instructions.
//
// TN (this file): dW = Gᵀ·[A1 | A2] over 16-row chunks (one MFMA k-step).  The chunk's three
// A planes are copied as rows into LDS ([plane][16 rows][352], 704-byte pitch ≡ 48 dwords mod
// 64) and read as the MFMA B operand by ds_read_b64_tr_b16 (a 16-lane group reads 4 rows x 16
// columns and receives them column-major: two reads give a lane its 8 consecutive rows of one
// column, conflict-free at this pitch).  G is formed and split on the fly as in gemm_x3.hip.
#include "gemm_common.hpp"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

namespace gnnmp {
namespace {

// ------------------------------------------------------------------ split image of an f32 matrix
// One thread per column pair of one row: hi / mid / lo words of the pair (zeros at columns >= F).
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                           int32_t F, uint16_t* __restrict__ img, int64_t ld,
                                                           int64_t ps, int32_t width) {
  const int hw = width >> 1;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * hw) return;
  const int64_t r = i / hw;
  const int c = 2 * (int)(i - r * hw);
  const float* xr = x + r * ldx;
  const float a = c < F ? xr[c] : 0.0f;
  const float b = c + 1 < F ? xr[c + 1] : 0.0f;
  uint32_t h, m, l;
  split3_pair(a, b, h, m, l);
  uint32_t* d = reinterpret_cast<uint32_t*>(img + r * ld + c);
  d[0] = h;
  d[ps >> 1] = m;
  d[ps] = l;
}

// ------------------------------------------------------------------ TN over a split image
constexpr int PT_ROWS = 16;               // rows per chunk = one MFMA k-step
constexpr int PT_AP = 352;                // LDS row pitch of an A chunk (bf16): 704 B ≡ 48 dwords mod 64
constexpr int PT_APL = PT_ROWS * PT_AP;   // one plane of a chunk
constexpr int PT_GP = 24;                 // G row pitch ([n][m], 12 dwords: conflict-free b128 reads)
constexpr int PT_GPL = 128 * PT_GP;
constexpr int PT_NP = 8;                  // 16-byte A pieces per thread per chunk (3·16·42 = 2016 <= 2048)
constexpr int PT_MAXLD = 336;             // widest image row the chunk layout holds (42 pieces)

// one transposed 4-row x 16-column read (lane i of each 16-lane group gets column i)
__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat_frag(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ floatx16 mfma6p(const bf16x8 (&x)[3], const bf16x8 (&y)[3], floatx16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[1], y[1], c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[2], y[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[1], y[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[0], c, 0, 0, 0);
  return c;
}

// Block: 4 waves (one per SIMD); wave w owns dW rows 32w .. +32 (G columns) x all KT k-tiles of
// the image width.  Rows: blockIdx.x·rows_per_block .. in chunks of 16, each LOADED from row
// min(start, M - 16) so every load is in bounds (the G mask zeroes rows outside the block).
// Staging per thread and chunk: PT_NP A pieces (one 16-byte buffer load + one ds_write_b128
// each) and one G slot (column n = tid mod 128, 8 consecutive rows) — h (MASK) or g values,
// G = (dz·P) ⊙ mask formed from a 2-slot LDS ring of dz rows (PROJ).
template <bool PROJ, bool MASK, int KT, bool GOUT>
__global__ __launch_bounds__(256) void gemm_tn_planes_kernel(TNArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Gt[2][3 * PT_GPL];
  __shared__ __attribute__((aligned(16))) uint16_t At[2][3 * PT_APL];
  __shared__ float Ps[MAXPROJ * 128];
  __shared__ float dzL[2][256];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ld = a.ap_ld;
  const int pr = ld >> 3;  // 16-byte pieces per image row
  const int64_t mbeg = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t mend = min(a.M, mbeg + a.rows_per_block);
  const int nch = mend > mbeg ? (int)((mend - mbeg + PT_ROWS - 1) / PT_ROWS) : 0;

  floatx16 acc[KT];
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

  // ---- A pieces of this thread (chunk-invariant): byte offsets in the image (relative to the
  //      chunk's first row) and in the LDS chunk.  Idle pieces re-load piece 0 into a pad slot
  //      (columns 336.. of plane 0, never part of a written dW column).
  const __amdgpu_buffer_rsrc_t arsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.ap), 0, (int)(3 * a.ap_ps * 2), 0x00020000);
  uint32_t goff[PT_NP], loff[PT_NP];
#pragma unroll
  for (int j = 0; j < PT_NP; ++j) {
    const int q = tid + 256 * j;
    const int per_plane = PT_ROWS * pr;
    const bool ok = q < 3 * per_plane;
    const int p = q / per_plane, rr = q - p * per_plane;
    const int row = rr / pr, c16 = rr - row * pr;
    goff[j] = ok ? (uint32_t)(((int64_t)p * a.ap_ps + (int64_t)row * ld + 8 * c16) * 2) : 0u;
    loff[j] = ok ? (uint32_t)((p * PT_APL + row * PT_AP + 8 * c16) * 2)
                 : (uint32_t)(((tid & 15) * PT_AP + PT_MAXLD + 8 * ((tid >> 4) & 1)) * 2);
  }

  // ---- G slot: column gn, rows 8·go .. +8 of the chunk
  const int gn = tid & 127, go = tid >> 7;
  const bool gcol = gn < a.Nr;
  const int gnc = gcol ? gn : 0;
  const float* gbase = MASK ? a.h + gnc : a.g + gnc;
  const int gld = MASK ? (int)a.ldh : (int)a.ldg;
  const float* g2base = a.g + gnc;  // the g form with MASK: g values beside h
  const int g2ld = (int)a.ldg;
  const int zr = (tid & 63) / MAXPROJ, zq = (tid & 63) % MAXPROJ;
  const int zqc = PROJ ? min(zq, a.nproj - 1) : 0;
  float pcol[MAXPROJ];
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) pcol[q] = 0.f;

  const int Mi = (int)a.M;
  auto ldbase = [&](int c) { return min((int)mbeg + c * PT_ROWS, Mi - PT_ROWS); };
  u32x4 ra[PT_NP];
  float rg[8], rg2[8];
  float rz = 0.f;
  auto load = [&](int c) {
    const int mb = ldbase(c);
    const int soff = mb * ld * 2;
#pragma unroll
    for (int j = 0; j < PT_NP; ++j) ra[j] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, (int)goff[j], soff, 0);
    if constexpr (MASK || !PROJ) {  // the dz form without a mask reads no G column
      uint32_t o = (uint32_t)((mb + 8 * go) * gld);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        rg[i] = gbase[o];
        o += (uint32_t)gld;
      }
    }
    if constexpr (MASK && !PROJ) {
      uint32_t o2 = (uint32_t)((mb + 8 * go) * g2ld);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        rg2[i] = g2base[o2];
        o2 += (uint32_t)g2ld;
      }
    }
    if constexpr (PROJ) rz = a.dz[(uint32_t)((ldbase(c + 1) + zr) * (int)a.lddz + zqc)];  // dz rows of chunk c + 1
  };

  float db = 0.f, dzs = 0.f;
  float dw2[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  auto store = [&](int c) {
    const int buf = c & 1;
    const int mb = ldbase(c);
    const int rlo = (int)mbeg + c * PT_ROWS - mb;  // valid loaded rows: [rlo, rhi)
    const int rhi = (int)mend - mb;
    if constexpr (PROJ) {  // dz ring slot of chunk c + 1 (slot read by G(c - 1): behind barrier c - 1)
      const int mb1 = ldbase(c + 1);
      const bool ok = tid < PT_ROWS * MAXPROJ && zq < a.nproj && zr >= (int)mbeg + (c + 1) * PT_ROWS - mb1 &&
                      zr < (int)mend - mb1;
      dzL[(c + 1) & 1][tid] = ok ? rz : 0.0f;
    }
    char* ab = reinterpret_cast<char*>(At[buf]);
#pragma unroll
    for (int j = 0; j < PT_NP; ++j) *reinterpret_cast<u32x4*>(ab + loff[j]) = ra[j];
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 8 * go + i;
      const bool ok = r >= rlo && r < rhi && gcol;
      float g;
      if constexpr (PROJ) {
        const float4 z = *reinterpret_cast<const float4*>(&dzL[buf][r * MAXPROJ]);
        g = z.x * pcol[0];
        g = fmaf(z.y, pcol[1], g);
        g = fmaf(z.z, pcol[2], g);
        g = fmaf(z.w, pcol[3], g);
        // staged dz rows are zero outside [rlo, rhi) and P is zero past Nr: no per-row masks
        if constexpr (MASK) {
          dw2[0] = fmaf(z.x, rg[i], dw2[0]);
          dw2[1] = fmaf(z.y, rg[i], dw2[1]);
          dw2[2] = fmaf(z.z, rg[i], dw2[2]);
          dw2[3] = fmaf(z.w, rg[i], dw2[3]);
        }
        const float zs = dzL[buf][r * MAXPROJ + (gn & (MAXPROJ - 1))];  // unconditional read + select:
        dzs += gn < MAXPROJ ? zs : 0.0f;                                 // no per-row branch
      } else {
        g = MASK ? rg2[i] : rg[i];
      }
      if constexpr (MASK) g = rg[i] > 0.0f ? g * a.hscale : 0.0f;
      if constexpr (!PROJ) g = ok ? g : 0.0f;
      db += g;
      if constexpr (GOUT) {
        if (a.gout && ok) a.gout[(int64_t)(mb + r) * a.ldgout + gn] = g;
      }
      e[i] = g;
    }
    uint32_t w[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) split3_pair(e[2 * j], e[2 * j + 1], w[j][0], w[j][1], w[j][2]);
    uint16_t* gd = Gt[buf] + gn * PT_GP + 8 * go;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      *reinterpret_cast<uint4*>(gd + p * PT_GPL) = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
  };

  // fragment addresses: G rows 32·wave + (lane & 31), k = 8·(lane >> 5); A (transposed reads)
  // lane 4q + p of 16-lane group g supplies row 8·(g >> 1) + q, columns 16·(g & 1) + 4p ..
  const int gfo = (32 * wave + (lane & 31)) * PT_GP + 8 * (lane >> 5);
  const int grp = lane >> 4, li = lane & 15;
  const int afo = (8 * (grp >> 1) + (li >> 2)) * PT_AP + 16 * (grp & 1) + 4 * (li & 3);
  auto afrag = [&](const uint16_t* base, int t, int p) {
    const uint16_t* q = base + p * PT_APL + t * 32;
    return cat_frag(tr_read(q), tr_read(q + 4 * PT_AP));
  };
  auto compute = [&](int c) {
    const int buf = c & 1;
    bf16x8 gf[3], af[2][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) gf[p] = *reinterpret_cast<const bf16x8*>(Gt[buf] + p * PT_GPL + gfo);
    const uint16_t* ab = At[buf] + afo;
#pragma unroll
    for (int p = 0; p < 3; ++p) af[0][p] = afrag(ab, 0, p);
    // tile t+1's fragment reads are issued before tile t's six MFMAs; the fences keep hipcc from
    // sinking them next to their use (it did: one exposed lgkmcnt(0) wait per tile)
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if (t + 1 < KT) {
#pragma unroll
        for (int p = 0; p < 3; ++p) af[(t + 1) & 1][p] = afrag(ab, t + 1, p);
      }
      __builtin_amdgcn_sched_barrier(0);
      acc[t] = mfma6p(gf, af[t & 1], acc[t]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if (nch > 0) {
    if constexpr (PROJ) {
#pragma unroll
      for (int q = 0; q < MAXPROJ; ++q) pcol[q] = (q < a.nproj && gcol) ? a.proj[q * a.Nr + gn] : 0.0f;
      const int mb0 = ldbase(0);
      const bool ok0 = tid < PT_ROWS * MAXPROJ && zq < a.nproj && zr >= (int)mbeg - mb0 && zr < (int)mend - mb0;
      dzL[0][tid] = ok0 ? a.dz[(int64_t)(mb0 + zr) * a.lddz + zqc] : 0.0f;
    }
    load(0);
    __syncthreads();  // Ps, dzL[0]
    for (int c = 0; c < nch; ++c) {
      store(c);  // buffers of chunk c - 2: last read before barrier c - 1
      __syncthreads();
      load(min(c + 1, nch - 1));
      compute(c);
    }
  }

  // ---- this block's partial dW (segment-major: dW1 = [Nr][k1] then dW2 = [Nr][k2])
  float* slab = a.slab + (int64_t)blockIdx.x * a.slab_stride;
  const int Kc = a.k1 + a.k2;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int kp = t * 32 + (lane & 31);  // image column
    const bool s1 = kp < a.k1;
    const bool s2 = kp >= a.ap_col2 && kp < a.ap_col2 + a.k2;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int64_t idx = s1 ? (int64_t)row * a.k1 + kp : (int64_t)a.Nr * a.k1 + (int64_t)row * a.k2 + (kp - a.ap_col2);
      if (row < a.Nr && (s1 || s2)) slab[idx] = acc[t][r];
    }
  }
  __syncthreads();
  // side sums of the two row octets combined in a fixed order through LDS (At[0] is free now)
  float* red = reinterpret_cast<float*>(&At[0][0]);
  constexpr int ns = 2 + MAXPROJ;
  red[(go * 128 + gn) * ns + 0] = db;
  red[(go * 128 + gn) * ns + 1] = dzs;
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) red[(go * 128 + gn) * ns + 2 + q] = dw2[q];
  __syncthreads();
  if (tid < 128 && tid < a.Nr) {
    float* side = slab + (int64_t)a.Nr * Kc;
    side[tid] = red[tid * ns] + red[(128 + tid) * ns];
    for (int q = 0; q < a.nproj; ++q)
      side[a.Nr + q * a.Nr + tid] = red[tid * ns + 2 + q] + red[(128 + tid) * ns + 2 + q];
  }
  if (PROJ && tid < a.nproj)
    slab[(int64_t)a.Nr * Kc + a.Nr + a.nproj * a.Nr + tid] = red[tid * ns + 1] + red[(128 + tid) * ns + 1];
}

template <bool PROJ, bool MASK, int KT>
void launch_tn_planes_k(const TNArgs& a, int nblk, hipStream_t st) {
  if (a.gout) gemm_tn_planes_kernel<PROJ, MASK, KT, true><<<nblk, 256, 0, st>>>(a);
  else gemm_tn_planes_kernel<PROJ, MASK, KT, false><<<nblk, 256, 0, st>>>(a);
}

template <int KT>
void launch_tn_planes_kt(const TNArgs& a, int nblk, hipStream_t st) {
  const bool proj = a.dz != nullptr, mask = a.h != nullptr;
  if (proj && mask) launch_tn_planes_k<true, true, KT>(a, nblk, st);
  else if (proj) launch_tn_planes_k<true, false, KT>(a, nblk, st);
  else if (mask) launch_tn_planes_k<false, true, KT>(a, nblk, st);
  else launch_tn_planes_k<false, false, KT>(a, nblk, st);
}

}  // namespace

bool tn_planes_ok(const TNArgs& a) {
  if (!a.ap || a.a_bf16 || a.h_bf16) return false;
  if (a.ap_ld % 16 || a.ap_ld > PT_MAXLD || a.ap_ld < 32) return false;
  if (a.k1 < 1 || a.k1 > a.ap_col2 || a.ap_col2 % 8 || a.ap_col2 + a.k2 > a.ap_ld) return false;
  if (a.ap_ps < a.M * (int64_t)a.ap_ld || (reinterpret_cast<uintptr_t>(a.ap) & 15)) return false;
  if (3 * a.ap_ps * 2 >= ((int64_t)1 << 31) || a.M < PT_ROWS) return false;
  const int64_t ldmax = std::max({a.h ? a.ldh : 0, a.g ? a.ldg : 0, a.dz ? a.lddz : 0});
  return (a.M + 32) * ldmax < ((int64_t)1 << 31);
}

void launch_tn_planes(const TNArgs& a, int nblk, hipStream_t st, int variant) {
  (void)variant;
  const int kt = (a.ap_ld + 31) / 32;
  if (kt <= 4) launch_tn_planes_kt<4>(a, nblk, st);
  else if (kt <= 6) launch_tn_planes_kt<6>(a, nblk, st);
  else if (kt <= 8) launch_tn_planes_kt<8>(a, nblk, st);
  else launch_tn_planes_kt<11>(a, nblk, st);
}

}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_split_planes_f32(const float* x, int64_t ldx, int64_t rows, int64_t F, void* img, int64_t ld,
                                           int64_t plane_stride, int64_t col0, int64_t width, gnn_stream_t stream) {
  if (rows < 0 || F < 0 || ldx < F || width < F || (width & 1) || (col0 & 1) || col0 < 0 || col0 + width > ld ||
      plane_stride < rows * ld || (plane_stride & 1) || (ld & 1))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad shapes (width >= F, even width / col0 / ld / plane_stride)");
  if (rows == 0 || width == 0) return GNN_OK;
  if (!x && F > 0) return fail(GNN_ERR_INVALID_ARG, __func__, "null x");
  if (!img || (reinterpret_cast<uintptr_t>(img) & 3)) return fail(GNN_ERR_INVALID_ARG, __func__, "null or unaligned image");
  const int64_t n = rows * (width / 2);
  split_planes_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(
      x, ldx, rows, (int32_t)F, static_cast<uint16_t*>(img) + col0, ld, plane_stride, (int32_t)width);
  return hip_check(hipGetLastError(), __func__);
}
