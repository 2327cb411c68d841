// Kernel lab (not part of the library): timing ablations of the split-image GEMMs on the SAGE
// layer-1 shape (M = 203,769 rows, image [3][M][336], 128 columns): the TN (dz form + mask) and
// the NT (bias + ReLU + dropout + projection), variants interleaved in one process, median of
// rounds.  Built by `make lab` (csrc/Makefile); run on the GPU box:  ./lab_gemm [rounds]
#define GNNMP_LAB 1
#include "../gemm_planes.hip"
#include "../gemm_ws.hip"

#include <algorithm>
#include <cstring>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

namespace gnnmp {
void set_last_error(const std::string&) {}
}

// Round-3 experiment kept here, not in the library: the split-image TN with every chunk operand
// (A planes, h, dz) copied into LDS rings by global_load_lds, two / three chunks ahead.  Bit-identical
// to gemm_tn_planes_kernel but slower: 164.7 vs 125.7 us (its DMA-only run 117.8 vs the
// register-staged "staging only" 120.6 us: the staging is bandwidth-, not latency-bound, and the
// DMA form overlaps worse with the MFMA chain).  profiles/r17_lab_gemm.txt.
namespace gnnmp {
namespace {
// The dz form with the h mask (PROJ && MASK, no G output): the SAGE hidden layer's weight gradient,
// the headline step's dominant kernel.  Same geometry, fragments, G slot, products, chunk order and
// side-sum order as gemm_tn_planes_kernel (results bit-identical), but every chunk operand reaches
// LDS by global_load_lds, with no register round trip and no VALU / ds_write per piece:
//   A: the chunk's three planes at the 704-byte row pitch of the transposed reads, 33 x 1 KB DMAs
//      (a lane's 16 bytes land in slot 64·i + lane of the chunk buffer, its source is the matching
//      image piece; a row's two pad pieces re-load its first piece, never read into a dW column);
//   h: the chunk's 16 x Nr f32 rows (8 x 1 KB);   dz: its 16 x 4 values (one dword DMA).
// The register-staged kernel holds one chunk in flight (its lab "staging only" run is as slow as
// the whole kernel: latency-bound on bytes in flight).  Here A runs two chunks ahead and h / dz
// three (rings of 3; G(c+1) is formed from h / dz during chunk c), 44 KB+ per CU in flight on top
// of the chunk being read.  The loop issues no other vector-memory operation: one counted vmcnt
// per chunk (this wave's NI DMAs of the newest group may stay in flight) orders the ring.  The
// DMAs are asm statements (M0 set in the statement), hidden from hipcc's waitcnt pass, which would
// otherwise drain them at the first LDS read after each barrier.
// LAB (csrc/lab/lab_gemm.hip only): bit 1 no MFMAs, bit 2 no G slots, bit 4 no fragment reads.
// GF: the g form (G read from a.g rows, no projection, no h mask: the GCN / GAT layer-1 weight
// gradient) — the h ring carries g's rows, no dz copy.
template <int KT, int LAB = 0, bool GF = false>
__global__ __launch_bounds__(256) void gemm_tn_planes_dma_kernel(TNArgs a) {
  constexpr int ACH = 3 * PT_APL * 2;          // one A chunk buffer: 33792 B = 33 x 1 KB
  constexpr int NA = ACH / 1024;
  constexpr int HCH = PT_ROWS * 128 * 4;       // one h chunk: 16 rows x 128 f32
  constexpr int NH = HCH / 1024;
  constexpr int NI = (NA + NH + 1 + 3) / 4;    // DMA instructions per wave per group (uniform: 11)
  constexpr int GCH = 3 * PT_GPL * 2;          // one G buffer (3 planes [n][m])
  constexpr int OA = 0, OH = OA + 3 * ACH, OZ = OH + 3 * HCH, OG = OZ + 3 * 256;
  constexpr int LDSB = OG + 2 * GCH;           // 163,584 B
  static_assert(ACH % 1024 == 0 && HCH % 1024 == 0 && LDSB <= 160 * 1024, "LDS layout");
  static_assert(6 * KT >= NI, "the DMA group issues in the chain's first slots");
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: DMA kinds / targets are wave-uniform
  const int ld = a.ap_ld;
  const int pr = ld >> 3;
  const int64_t mbeg = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t mend = min(a.M, mbeg + a.rows_per_block);
  const int nch = mend > mbeg ? (int)((mend - mbeg + PT_ROWS - 1) / PT_ROWS) : 0;
  const int Mi = (int)a.M;
  auto ldbase = [&](int c) __attribute__((always_inline)) { return min((int)mbeg + c * PT_ROWS, Mi - PT_ROWS); };
  const int clast = max(nch - 1, 0);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);

  floatx16 acc[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  // ---- DMA sources: instruction I = wave + 4j of a group; this lane's byte offset from the
  //      chunk's first row of the instruction's operand
  auto a_off = [&](int I) __attribute__((always_inline)) {
    const int q = 64 * I + lane;
    const int p = q / (PT_ROWS * (PT_AP / 8)), rr = q - p * (PT_ROWS * (PT_AP / 8));
    const int row = rr / (PT_AP / 8), pc = rr - row * (PT_AP / 8);
    return (uint32_t)(((int64_t)p * a.ap_ps + (int64_t)row * ld) * 2) + (pc < pr ? 16u * pc : 0u);
  };
  const int hcol = min(4 * (lane & 31), (int)a.Nr - 4);
  const int ldhg = GF ? (int)a.ldg : (int)a.ldh;  // the h ring's rows: h, or g in the g form
  constexpr int NDUP0 = GF ? NA + NH : NA + NH + 1;  // first count-padding instruction
  uint32_t voff[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int I = wave + 4 * j;
    if (I < NA) voff[j] = a_off(I);
    else if (I < NA + NH) voff[j] = (uint32_t)(((2 * (I - NA) + (lane >> 5)) * ldhg + hcol) * 4);
    else if (!GF && I == NA + NH) voff[j] = (uint32_t)(((lane >> 2) * (int)a.lddz + min(lane & 3, a.nproj - 1)) * 4);
    else voff[j] = a_off(I - NDUP0);  // count padding: a duplicate of an A instruction (same bytes, same slot)
  }
  // prologue group of h(0) / dz(0) alone: 3 per wave (I' = wave + 4j: h 0..7, dz 8, duplicates of h 0..2)
  uint32_t voff0[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int I = wave + 4 * j;
    const int k = I < NH ? I : (!GF && I == NH) ? 0 : I - NH - (GF ? 0 : 1);
    voff0[j] = (!GF && I == NH) ? (uint32_t)(((lane >> 2) * (int)a.lddz + min(lane & 3, a.nproj - 1)) * 4)
                                : (uint32_t)(((2 * k + (lane >> 5)) * ldhg + hcol) * 4);
  }
  auto glds16 = [](const void* src, uint32_t dst) __attribute__((always_inline)) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst)));
  };
  auto glds4 = [](const void* src, uint32_t dst) __attribute__((always_inline)) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst)));
  };
  auto wait_vm = [](auto nc) __attribute__((always_inline)) {  // vmcnt(N) alone (gfx9 encoding)
    constexpr int N = decltype(nc)::value;
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  };
  const char* const apb = reinterpret_cast<const char*>(a.ap);
  const char* const hb = reinterpret_cast<const char*>(GF ? a.g : a.h);
  const char* const zb = reinterpret_cast<const char*>(a.dz);
  // DMA j of group g(c) = {A(c + 2) -> A buffer (c + 2) % 3, h / dz(c + 3) -> buffers (c + 3) % 3}.
  // The instruction's operand is wave-uniform; its parameters are chosen here, at kernel scope (a
  // select among captured values inside the lambda becomes a load from a selected closure address,
  // which keeps the closure in scratch)
  uint64_t sbase[NI];
  int srb[NI], sofs[NI], sstr[NI], sdst[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int I = wave + 4 * j;
    const bool isA = I < NA || I >= NDUP0, isZ = !GF && I == NA + NH;
    sbase[j] = isA ? (uint64_t)(uintptr_t)apb : isZ ? (uint64_t)(uintptr_t)zb : (uint64_t)(uintptr_t)hb;
    srb[j] = isA ? ld * 2 : isZ ? (int)a.lddz * 4 : ldhg * 4;
    sofs[j] = isA ? 2 : 3;
    sstr[j] = isA ? ACH : isZ ? 256 : HCH;
    sdst[j] = isA ? OA + (I < NA ? I : I - NDUP0) * 1024 : isZ ? OZ : OH + (I - NA) * 1024;
  }
  const bool zwave = wave == (NA + NH) % 4;  // the wave whose last DMA is dz's dword copy
  auto dma = [&](int j, int c) __attribute__((always_inline)) {
    const char* src = reinterpret_cast<const char*>(sbase[j]) + (int64_t)ldbase(min(c + sofs[j], clast)) * srb[j] + voff[j];
    const uint32_t dst = lds0 + (uint32_t)(sdst[j] + ((c + sofs[j]) % 3) * sstr[j]);
    if (!GF && j == (NA + NH) / 4 && zwave) glds4(src, dst);
    else glds16(src, dst);
  };
  auto sync = [&]() __attribute__((always_inline)) {  // the ring's barrier: own LDS writes done, then every wave's
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- G slot: column gn, rows 8·go .. +8 of the chunk (the register-staged kernel's)
  const int gn = tid & 127, go = tid >> 7;
  const bool gcol = gn < a.Nr;
  float pcol[MAXPROJ];
#pragma unroll
  for (int q = 0; q < MAXPROJ; ++q) pcol[q] = (q < a.nproj && gcol) ? a.proj[q * a.Nr + gn] : 0.0f;
  float db = 0.f, dzs = 0.f;
  float dw2[MAXPROJ] = {0.f, 0.f, 0.f, 0.f};
  float e[8], hv[8];
  uint32_t w[4][3];
  float4 zv[8];
  float zsv[8];
  // rows i0, i0 + 1 of the slot for chunk k: h and dz from the LDS rings (dz rows outside the
  // block's range read as zero: G, dzᵀh and Σdz need no other row mask)
  auto hz_read = [&](int k, int i0) __attribute__((always_inline)) {
    const int mb = ldbase(k);
    const float* hs = reinterpret_cast<const float*>(smem + OH + (k % 3) * HCH);
    const float* zs = reinterpret_cast<const float*>(smem + OZ + (k % 3) * 256);
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i) {
      const int r = 8 * go + i;
      const bool ok = r >= (int)mbeg + k * PT_ROWS - mb && r < (int)mend - mb;
      hv[i] = hs[r * 128 + (gcol ? gn : 0)];
      if constexpr (GF) {  // g rows outside the block's range: zero G
        hv[i] = ok && gcol ? hv[i] : 0.f;
        continue;
      }
      const float4 z = *reinterpret_cast<const float4*>(zs + r * MAXPROJ);
      const float zs1 = zs[r * MAXPROJ + (gn & (MAXPROJ - 1))];
      zv[i] = ok ? z : make_float4(0.f, 0.f, 0.f, 0.f);
      zsv[i] = ok ? zs1 : 0.f;
    }
  };
  auto g_row = [&](int i, int half) __attribute__((always_inline)) {
    if constexpr (GF) {
      if (half == 0) e[i] = hv[i];
      else db += e[i];
      return;
    }
    if (half == 0) {
      const float4 z = zv[i];
      float g = z.x * pcol[0];
      g = fmaf(z.y, pcol[1], g);
      g = fmaf(z.z, pcol[2], g);
      e[i] = fmaf(z.w, pcol[3], g);
      dw2[0] = fmaf(z.x, hv[i], dw2[0]);
      dw2[1] = fmaf(z.y, hv[i], dw2[1]);
      dw2[2] = fmaf(z.z, hv[i], dw2[2]);
      dw2[3] = fmaf(z.w, hv[i], dw2[3]);
      return;
    }
    dzs += gn < MAXPROJ ? zsv[i] : 0.0f;
    const float g = hv[i] > 0.0f ? e[i] * a.hscale : 0.0f;
    db += g;
    e[i] = g;
  };
  auto split_half = [&](int j, int half) __attribute__((always_inline)) {
    float& x0 = e[2 * j];
    float& x1 = e[2 * j + 1];
    if (half == 0) {
      const uint32_t h = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v_t){x0, x1}, bf16x2v_t));
      w[j][0] = h;
      x0 -= __uint_as_float(h << 16);
      x1 -= __uint_as_float(h & 0xffff0000u);
    } else {
      const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v_t){x0, x1}, bf16x2v_t));
      w[j][1] = m;
      const float y0 = x0 - __uint_as_float(m << 16);
      const float y1 = x1 - __uint_as_float(m & 0xffff0000u);
      w[j][2] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v_t){y0, y1}, bf16x2v_t));
    }
  };
  auto g_put = [&](int k) __attribute__((always_inline)) {
    uint16_t* gd = reinterpret_cast<uint16_t*>(smem + OG + (k & 1) * GCH) + gn * PT_GP + 8 * go;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      *reinterpret_cast<uint4*>(gd + p * PT_GPL) = make_uint4(w[0][p], w[1][p], w[2][p], w[3][p]);
  };
  // slot k of chunk c's chain: the DMA group g(c), then G(c + 1) from the h / dz rings
  constexpr int U_HZ = NI, U_G = U_HZ + 4, U_S = U_G + 16, U_P = U_S + 8, NU = U_P + 1;
  auto unit = [&](int k, int c) __attribute__((always_inline)) {
    if (k < U_HZ) return;  // the DMAs: issued by the chain itself (compile-time j)
    if (LAB & 2) return;
    else if (k < U_G) hz_read(c + 1, 2 * (k - U_HZ));
    else if (k < U_S) g_row((k - U_G) >> 1, (k - U_G) & 1);
    else if (k < U_P) split_half((k - U_S) >> 1, (k - U_S) & 1);
    else g_put(c + 1);
  };

  const int gfo = (32 * wave + (lane & 31)) * PT_GP + 8 * (lane >> 5);
  const int grp = lane >> 4, li = lane & 15;
  const int afo = (8 * (grp >> 1) + (li >> 2)) * PT_AP + 16 * (grp & 1) + 4 * (li & 3);
  auto afrag = [&](const uint16_t* base, int t, int p) __attribute__((always_inline)) {
    const uint16_t* q = base + p * PT_APL + t * 32;
    return cat_frag(tr_read(q), tr_read(q + 4 * PT_AP));
  };
#define PD_FENCE __builtin_amdgcn_sched_barrier(0)
  auto compute = [&](int c) __attribute__((always_inline)) {
    const uint16_t* gt = reinterpret_cast<const uint16_t*>(smem + OG + (c & 1) * GCH);
    bf16x8 gf[3], af[2][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) gf[p] = *reinterpret_cast<const bf16x8*>(gt + p * PT_GPL + gfo);
    const uint16_t* ab = reinterpret_cast<const uint16_t*>(smem + OA + (c % 3) * ACH) + afo;
#pragma unroll
    for (int p = 0; p < 3; ++p) af[0][p] = afrag(ab, 0, p);
    constexpr int pa[6] = {1, 2, 0, 1, 0, 0}, pb[6] = {1, 0, 2, 0, 1, 0};  // small terms first
    static_for<KT>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t + 1 < KT && !(LAB & 4)) {
#pragma unroll
        for (int p = 0; p < 3; ++p) af[(t + 1) & 1][p] = afrag(ab, t + 1, p);
      }
      static_for<6>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        PD_FENCE;
        if constexpr (!(LAB & 1))
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf[pa[m]], af[(LAB & 4) ? 0 : (t & 1)][pb[m]], acc[t], 0, 0, 0);
        PD_FENCE;
        if constexpr (6 * t + m < U_HZ) dma(6 * t + m, c);
        else if constexpr (6 * t + m < NU) unit(6 * t + m, c);
      });
      PD_FENCE;
    });
#pragma unroll
    for (int u = max(6 * KT, U_HZ); u < NU; ++u) unit(u, c);  // narrow images: the slots past the MFMAs
    if constexpr ((LAB & 1) != 0) {
#pragma unroll
      for (int t = 0; t < KT; ++t) acc[t][0] += (float)gf[0][0] + (float)af[0][0][0] + (float)af[1][1][1];
    }
  };
#undef PD_FENCE

  if (nch > 0) {
    wait_vm(std::integral_constant<int, 0>{});  // the projection loads: nothing compiler-known in flight below
    // prologue: h / dz(0) alone, then groups g(-2) = {A(0), h(1)}, g(-1) = {A(1), h(2)}
    {
      const int mb = ldbase(0);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int I = wave + 4 * j;
        if (!GF && I == NH) glds4(zb + (int64_t)mb * a.lddz * 4 + voff0[j], lds0 + (uint32_t)OZ);
        else glds16(hb + (int64_t)mb * ldhg * 4 + voff0[j],
                    lds0 + (uint32_t)(OH + (I < NH ? I : I - NH - (GF ? 0 : 1)) * 1024));
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) dma(j, -2);
#pragma unroll
    for (int j = 0; j < NI; ++j) dma(j, -1);
    wait_vm(std::integral_constant<int, 2 * NI>{});  // h / dz(0)
    sync();
    hz_read(0, 0); hz_read(0, 2); hz_read(0, 4); hz_read(0, 6);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      g_row(i, 0);
      g_row(i, 1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      split_half(j, 0);
      split_half(j, 1);
    }
    g_put(0);
    wait_vm(std::integral_constant<int, NI>{});  // g(-2): A(0), h / dz(1)
    sync();
    for (int c = 0; c < nch; ++c) {
      compute(c);  // + g(c) and G(c + 1)
      wait_vm(std::integral_constant<int, NI>{});  // g(c - 1): A(c + 1), h / dz(c + 2)
      sync();
    }
    wait_vm(std::integral_constant<int, 0>{});  // no DMA may outlive the block's LDS
    sync();
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
  // side sums of the two row octets in a fixed order through LDS (the A ring is free now)
  float* red = reinterpret_cast<float*>(smem + OA);
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
  if (tid < a.nproj)
    slab[(int64_t)a.Nr * Kc + a.Nr + a.nproj * a.Nr + tid] = red[tid * ns + 1] + red[(128 + tid) * ns + 1];
}

}  // namespace
}  // namespace gnnmp

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

static float* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  std::mt19937 g(seed);
  std::normal_distribution<float> d(0.f, scale);
  for (auto& v : h) v = d(g);
  float* p;
  CK(hipMalloc(&p, n * sizeof(float)));
  CK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return p;
}

using namespace gnnmp;

// MFMA issue microbenchmark: one wave per SIMD (256 x 256 threads), 24·iters
// v_mfma_f32_32x32x16_bf16 per wave on random data, as NCH interleaved accumulator chains;
// shader clocks (s_memtime) and 100 MHz ticks (s_memrealtime) of wave 0 of block 0.
template <int NCH>
__global__ __launch_bounds__(256) void mfma_chain_kernel(const uint4* in, float* out, int iters,
                                                         unsigned long long* clk) {
  const bf16x8 x = __builtin_bit_cast(bf16x8, in[threadIdx.x]);
  const bf16x8 y = __builtin_bit_cast(bf16x8, in[256 + threadIdx.x]);
  floatx16 acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 24 / NCH; ++k)
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, acc[c], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c][0] + acc[c][15];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

template <int NCH>
void mfma_probe(const uint4* in, float* out, unsigned long long* clk) {
  const int iters = 2000;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  mfma_chain_kernel<NCH><<<256, 256>>>(in, out, iters, clk);
  CK(hipEventRecord(e0));
  mfma_chain_kernel<NCH><<<256, 256>>>(in, out, iters, clk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
  const double n = 24.0 * iters;
  std::printf("MFMA chains=%d: %.1f us, %.1f shader cycles / MFMA, clock %.2f GHz, %.0f TF/s bf16\n", NCH,
              ms * 1e3, h[0] / n, h[0] / (h[1] * 10.0), n * 1024 * 32768.0 / (ms * 1e-3) / 1e12);
}

template <int LAB>
void tn(const TNArgs& a, const NTArgs&, const uint4*, int nblk, int) {
  gemm_tn_planes_kernel<true, true, 11, false, LAB><<<nblk, 256>>>(a);
}
template <int LAB>
void tnd(const TNArgs& a, const NTArgs&, const uint4*, int nblk, int) {
  gemm_tn_planes_dma_kernel<11, LAB><<<nblk, 256>>>(a);
}
static TNArgs g_gcn;  // the GCN layer-1 TN: dW = Gᵀ·x over x's 176-wide image, Nr = 64, g form
template <int LAB>
void tng(const TNArgs&, const NTArgs&, const uint4*, int nblk, int) {
  gemm_tn_planes_kernel<false, false, 6, false, LAB><<<nblk, 256>>>(g_gcn);
}
template <int LAB>
void tngk(const TNArgs&, const NTArgs&, const uint4*, int nblk, int) {
  gemm_tn_planes_kernel<false, false, 6, false, LAB, 2><<<nblk, 256>>>(g_gcn);
}
template <int LAB>
void tngk8(const TNArgs&, const NTArgs&, const uint4*, int nblk, int) {  // 8 waves: 2 row groups x 4 k-groups
  gemm_tn_planes_kernel<false, false, 6, false, LAB, 4, 8><<<nblk, 512>>>(g_gcn);
}
template <int LAB>
void tngd(const TNArgs&, const NTArgs&, const uint4*, int nblk, int) {
  gemm_tn_planes_dma_kernel<6, LAB, true><<<nblk, 256>>>(g_gcn);
}
template <int EPI>
void nte(const TNArgs&, const NTArgs& a, const uint4* img, int, int ntiles) {
  gemm_nt_planes_kernel<21, EPI, 0><<<256, 256>>>(a, img, ntiles);
}
template <int LAB>
void nt(const TNArgs&, const NTArgs& a, const uint4* img, int, int ntiles) {
  gemm_nt_planes_kernel<21, WS_BIAS | WS_RELU | WS_DROP | WS_PROJ, LAB><<<256, 256>>>(a, img, ntiles);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 9;
  const int64_t M = 203769, F = 166, LD = 336, NR = 128;
  float* x = dev_rand(M * 2 * F, 1.f, 1);
  uint16_t* img;
  CK(hipMalloc(&img, 3 * M * LD * 2));
  gnn_split_planes_f32(x, 2 * F, M, F, img, LD, M * LD, 0, 168, nullptr);
  gnn_split_planes_f32(x + F, 2 * F, M, F, img, LD, M * LD, 168, 168, nullptr);
  float* h = dev_rand(M * NR, 1.f, 2);
  float* dz = dev_rand(M * 4, 1e-3f, 3);
  float* proj = dev_rand(4 * NR, 1.f, 4);
  float* w1 = dev_rand(NR * F, 0.08f, 5);
  float* w2 = dev_rand(NR * F, 0.08f, 6);
  float* bias = dev_rand(NR, 0.1f, 7);
  float *c, *z;
  CK(hipMalloc(&c, M * NR * 4));
  CK(hipMalloc(&z, M * 4 * 4));
  const int nblk = 256;
  const int64_t stride = (NR * 332 + NR + 4 * NR + 4 + 63) / 64 * 64;
  float* slab;
  CK(hipMalloc(&slab, nblk * stride * 4));
  TNArgs a{};
  a.M = M; a.Nr = NR; a.dz = dz; a.lddz = 4; a.proj = proj; a.nproj = 4; a.h = h; a.ldh = NR; a.hscale = 2.f;
  a.k1 = F; a.k2 = F; a.slab = slab; a.slab_stride = stride;
  a.rows_per_block = ceil_div(ceil_div(M, 32), nblk) * 32;
  a.ap = img; a.ap_ld = LD; a.ap_col2 = 168; a.ap_ps = M * LD;
  NTArgs n{};
  n.M = M; n.Nc = NR; n.k1 = F; n.k2 = F; n.w1 = w1; n.w2 = w2; n.ldw1 = F; n.ldw2 = F; n.c = c; n.ldc = NR;
  n.bias = bias; n.relu = 1; n.dropout = 1; n.keep_thresh = (uint32_t)(0.5 * 16777216.0); n.drop_scale = 2.f;
  n.seed = 1234; n.proj = proj; n.nproj = 4; n.z = z; n.ldz = 4;
  n.ap = img; n.ap_ld = LD; n.ap_col2 = 168; n.ap_ps = M * LD;
  uint4* bimg;
  CK(hipMalloc(&bimg, 21 * 3 * 256 * 16));
  ws_prep_kernel<<<21, 256>>>(n, bimg, 21, nullptr, 0, 168);
  const int ntiles = (int)ceil_div(M, 32);
  {  // GCN layer 1: x alone at 176-wide rows, G [M, 64]
    uint16_t* img2;
    CK(hipMalloc(&img2, 3 * M * 176 * 2));
    gnn_split_planes_f32(x, 2 * F, M, F, img2, 176, M * 176, 0, 176, nullptr);
    g_gcn = TNArgs{};
    g_gcn.M = M; g_gcn.Nr = 64; g_gcn.g = dev_rand(M * 64, 1.f, 11); g_gcn.ldg = 64;
    g_gcn.k1 = F; g_gcn.k2 = 0; g_gcn.hscale = 1.f;
    g_gcn.slab = slab; g_gcn.slab_stride = (64 * F + 64 + 63) / 64 * 64;
    g_gcn.rows_per_block = a.rows_per_block;
    g_gcn.ap = img2; g_gcn.ap_ld = 176; g_gcn.ap_col2 = 168; g_gcn.ap_ps = M * 176;
  }
  struct V { const char* name; void (*f)(const TNArgs&, const NTArgs&, const uint4*, int, int); std::vector<float> t; };
  std::vector<V> vs = {
      {"TN production", tn<0>, {}}, {"TN no MFMA", tn<1>, {}}, {"TN no staging", tn<2>, {}},
      {"TN no frag reads", tn<4>, {}}, {"TN no barrier", tn<8>, {}}, {"TN MFMA+frags", tn<2 | 8>, {}},
      {"TN MFMA only", tn<2 | 4 | 8>, {}}, {"TN staging only", tn<1 | 4>, {}},
      {"GCN TN production", tng<0>, {}}, {"GCN TN split-K", tngk<0>, {}}, {"GCN TN 8 waves", tngk8<0>, {}},
      {"GCN TN 8w staging", tngk8<1 | 4>, {}}, {"GCN TN dma", tngd<0>, {}}, {"GCN TN staging only", tng<1 | 4>, {}},
      {"GCN TN dma DMA only", tngd<1 | 2 | 4>, {}},
      {"TN dma", tnd<0>, {}}, {"TN dma no MFMA", tnd<1>, {}}, {"TN dma no G", tnd<2>, {}},
      {"TN dma no frags", tnd<4>, {}}, {"TN dma DMA only", tnd<1 | 2 | 4>, {}},
      {"NT production", nt<0>, {}}, {"NT no MFMA", nt<1>, {}}, {"NT no epilogue", nt<2>, {}},
      {"NT no staging", nt<4>, {}}, {"NT no mid barrier", nt<8>, {}}, {"NT MFMA+frags only", nt<2 | 4 | 8>, {}},
      {"NT epilogue only", nt<1 | 4>, {}},
      {"NT no dropout", nte<WS_BIAS | WS_RELU | WS_PROJ>, {}}, {"NT no projection", nte<WS_BIAS | WS_RELU | WS_DROP>, {}},
      {"NT bias+relu only", nte<WS_BIAS | WS_RELU>, {}}};
  {
    std::vector<uint16_t> hb(512 * 8);  // random bf16 operands (truncated normal floats: no NaN)
    std::mt19937 g(9);
    std::normal_distribution<float> d(0.f, 1.f);
    for (auto& v : hb) {
      const float f = d(g);
      uint32_t u;
      std::memcpy(&u, &f, 4);
      v = (uint16_t)(u >> 16);
    }
    uint4* in;
    CK(hipMalloc(&in, hb.size() * 2));
    CK(hipMemcpy(in, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    float* out;
    unsigned long long* clk;
    CK(hipMalloc(&out, 256 * 256 * 4));
    CK(hipMalloc(&clk, 16));
    mfma_probe<1>(in, out, clk);
    mfma_probe<2>(in, out, clk);
    mfma_probe<4>(in, out, clk);
    mfma_probe<1>(in, out, clk);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  {  // the DMA-ring TN against the register-staged one: the same products in the same order
    const size_t nsl = (size_t)nblk * stride;
    std::vector<float> r0(nsl), r1(nsl);
    CK(hipMemset(slab, 0, nsl * 4));
    tn<0>(a, n, bimg, nblk, ntiles);
    CK(hipMemcpy(r0.data(), slab, nsl * 4, hipMemcpyDeviceToHost));
    CK(hipMemset(slab, 0, nsl * 4));
    tnd<0>(a, n, bimg, nblk, ntiles);
    CK(hipMemcpy(r1.data(), slab, nsl * 4, hipMemcpyDeviceToHost));
    size_t ndiff = 0;
    double md = 0;
    for (size_t i = 0; i < nsl; ++i)
      if (std::memcmp(&r0[i], &r1[i], 4)) {
        ++ndiff;
        md = std::max(md, (double)std::fabs(r0[i] - r1[i]));
      }
    std::printf("TN dma vs production: %zu of %zu slab words differ (max |diff| %g)\n", ndiff, nsl, md);
    CK(hipMemset(slab, 0, nsl * 4));
    tng<0>(a, n, bimg, nblk, ntiles);
    CK(hipMemcpy(r0.data(), slab, nsl * 4, hipMemcpyDeviceToHost));
    CK(hipMemset(slab, 0, nsl * 4));
    tngd<0>(a, n, bimg, nblk, ntiles);
    CK(hipMemcpy(r1.data(), slab, nsl * 4, hipMemcpyDeviceToHost));
    ndiff = 0;
    md = 0;
    for (size_t i = 0; i < nsl; ++i)
      if (std::memcmp(&r0[i], &r1[i], 4)) {
        ++ndiff;
        md = std::max(md, (double)std::fabs(r0[i] - r1[i]));
      }
    std::printf("GCN TN dma vs production: %zu of %zu slab words differ (max |diff| %g)\n", ndiff, nsl, md);
    CK(hipMemset(slab, 0, nsl * 4));
    tngk<0>(a, n, bimg, nblk, ntiles);
    CK(hipMemcpy(r1.data(), slab, nsl * 4, hipMemcpyDeviceToHost));
    ndiff = 0;
    for (size_t i = 0; i < nsl; ++i) ndiff += std::memcmp(&r0[i], &r1[i], 4) != 0;
    std::printf("GCN TN split-K vs production: %zu of %zu slab words differ\n", ndiff, nsl);
    CK(hipMemset(slab, 0, nsl * 4));
    tngk8<0>(a, n, bimg, nblk, ntiles);
    CK(hipMemcpy(r1.data(), slab, nsl * 4, hipMemcpyDeviceToHost));
    ndiff = 0;
    md = 0;
    for (size_t i = 0; i < nsl; ++i)
      if (std::memcmp(&r0[i], &r1[i], 4)) {
        ++ndiff;
        md = std::max(md, (double)std::fabs(r0[i] - r1[i]));
      }
    std::printf("GCN TN 8 waves vs production: %zu of %zu slab words differ (max |diff| %g; dW bit-exact, the side sums' order)\n",
                ndiff, nsl, md);
  }
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      v.f(a, n, bimg, nblk, ntiles);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) v.f(a, n, bimg, nblk, ntiles);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms * 1000.f / 5);
    }
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    std::printf("%-20s %8.1f us (min %.1f)\n", v.name, v.t[v.t.size() / 2], v.t[0]);
  }
  return 0;
}
