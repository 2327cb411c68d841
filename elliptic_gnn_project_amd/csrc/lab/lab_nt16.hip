// Kernel lab (not part of the library): the half-pair NT on the SAGE layer-1 shape (M = 203,769,
// [agg | x] = 336-wide half-pair image, N = 128, bias + ReLU + dropout + projection): the 32-row
// form (gemm_nt_h2_kernel) against the 16-row ring form (gemm_nt_h2r_kernel), with ablations,
// and a plain stream of the same bytes for reference.  Timings: variants interleaved, median.
//   make -C elliptic_gnn_project_amd/csrc labnt16 && elliptic_gnn_project_amd/_lab/lab_nt16
#define GNNMP_LAB 1
#include "../gemm_planes.hip"
#include "../gemm_ws.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

namespace gnnmp {
void set_last_error(const std::string&) {}
}

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

namespace gnnmp {
namespace {
typedef float floatx4 __attribute__((ext_vector_type(4)));
// The 16-row ring form of the half-pair NT (round 5 experiment; measured slower in the step than
// gemm_nt_h2_kernel: 93.3 vs 90.1 us, profiles/r26_ab_nt.txt — kept here, not in the library).
// ---------------------------------------------------------------- half-pair NT, 16-row ring form (K7h-r)
// The same product as gemm_nt_h2_kernel, laid out for TWO waves per SIMD so the hardware overlaps
// one wave's epilogue / staging with the other's MFMA chain (the 32-row form holds 252 AGPRs of B
// in one wave per SIMD and interleaves everything by hand: lab r19 "no MFMA" 74.6 of 89.9 us,
// i.e. its memory and epilogue work does not hide under the 42 us chain).
//   * 16-row tiles, v_mfma_f32_16x16x32_f16; 256-thread blocks, TWO per CU (grid 2 x CUs, 256
//     registers per wave: __launch_bounds__(256, 2)).  Wave w owns columns 32w .. +32 as two
//     16-column halves; its B fragments — planes hi and lo only, read from the 3-plane B image
//     (ws_prep_h2_cols) — stay in AGPRs: NK 32-deep k-steps x 2 planes x 2 halves x 4 = 176 (NK 11).
//   * two accumulators per half instead of the hi' = 2^11 hi plane:
//       x  += A_hi·B_lo + A_lo·B_hi,    hh += A_hi·B_hi,    C = (2^11 hh + x) · 2^(e_n - 11 - ap_exp)
//     (= the 3-product form's sum, two chains per half: four independent MFMA chains per wave).
//   * A staged by an LDS-DMA ring (global_load_lds_dwordx4, as gemm_nt_img16_kernel): NBUF = 3
//     tile buffers of [plane 2][k-step NK][16 rows x 64 B] (1 KB blocks, the k-quarter of row r
//     at slot q ^ ((r >> 2) & 3): conflict-free ds_read_b128 of the A fragments), two tiles in
//     flight per block, counted vmcnt waits, one s_barrier per tile.  Columns past the image row
//     (k >= ld in the last k-step) load an in-row value; their B fragments are zero.
//   * epilogue straight from the accumulators: bias, ReLU, counter-hash dropout (keep_elem of
//     row·Nc + col, bit for bit), dword C stores (4 rows x 64 B per instruction), and the
//     projection z = h·Pᵀ: per-lane partials over the lane's 2 columns, a reduce-and-split
//     butterfly over the 16 lanes of a row group, per-wave partials in LDS summed over the 4
//     column blocks in a fixed order one tile later (one z store per wave per tile).
// LAB: bit 1 no MFMAs, 2 no epilogue, 4 no DMA,
// 8 the A-fragment prefetch pinned by scheduling fences (spills 16 VGPRs of B: not the default).
constexpr int H2R_ROWS = 16;
template <bool FIRST>
__device__ __forceinline__ void h2r_mfma(floatx4& acc, const f16x8& x, const f16x8& b) {
#if GNNMP_H2R_ASM
  if constexpr (FIRST) asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=v"(acc) : "v"(x), "a"(b));
  else asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(x), "a"(b));
#else
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, b, FIRST ? floatx4{0.f, 0.f, 0.f, 0.f} : acc, 0, 0, 0);
#endif
}
__device__ __forceinline__ void h2r_mfma_end(floatx4& a0, floatx4& a1, floatx4& a2, floatx4& a3) {
#if GNNMP_H2R_ASM
  asm volatile("s_nop 15\n\ts_nop 7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
#endif
}

template <int NK, int EPI, int LAB = 0>
__global__ __launch_bounds__(256, 2) void gemm_nt_h2r_kernel(NTArgs a, const uint4* __restrict__ bimg,
                                                             const float* __restrict__ colscale, int ntiles) {
  constexpr int NBUF = 3;
  constexpr int KB = 1024;                       // one (plane, k-step) block: 16 rows x 32 f16
  constexpr int NBLK = 2 * NK;                   // DMA blocks per tile
  constexpr int ABUF = NBLK * KB;
  constexpr int QW = (NBLK + 3) / 4;             // DMAs per wave per tile (uniform: vmcnt accounting)
  constexpr int SCR = NBUF * ABUF;               // 1 KB target of the count-padding DMAs
  constexpr int ZP0 = SCR + KB;                  // two [4 waves][16 rows][4] f32 projection partials
  constexpr int ZPB = 4 * H2R_ROWS * MAXPROJ * 4;
  constexpr int PL0 = ZP0 + 2 * ZPB;             // the projection P [MAXPROJ][BN] f32 (read per tile)
  constexpr int LDSB = PL0 + MAXPROJ * BN * 4;
  constexpr bool PROJ = (EPI & WS_PROJ) != 0;
  constexpr int S = 8 + 1;                       // stores per wave per tile: 8 C dwords + 1 z
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t M = a.M;
  const int Nc = a.Nc;
  const int ld = a.ap_ld;
  const uint64_t seed = a.seed_ptr ? (*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;
  int t = blockIdx.x;
  if (t >= ntiles) return;
  const int G = gridDim.x;
  const bool active = 32 * wave < Nc;            // wave-uniform: columns past N multiply zeros

  // ---- stationary B (planes hi = 1, lo = 2 of the 32-row form's image): lane l holds column
  //      32·wave + 16·half + (l & 15), k = 32 s + 8 (l >> 4) .. +8 = image k-step 2s + (l >> 5),
  //      slot half (l >> 4) & 1; k-steps past the image (ld / 16 of them) are zero
  const int nks16 = ld / 16;
  f16x8 bh[NK][2], bl[NK][2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const int slot = 2 * (32 * wave + 16 * hf + (lane & 15)) + ((lane >> 4) & 1);
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      const int s16 = 2 * s + (lane >> 5);
      const bool ok = s16 < nks16;
      const int sc = ok ? s16 : 0;
      const uint4 h = bimg[(sc * 3 + 1) * 256 + slot], l = bimg[(sc * 3 + 2) * 256 + slot];
      bh[s][hf] = __builtin_bit_cast(f16x8, ok ? h : make_uint4(0u, 0u, 0u, 0u));
      bl[s][hf] = __builtin_bit_cast(f16x8, ok ? l : make_uint4(0u, 0u, 0u, 0u));
    }
  }
  // ---- epilogue constants: this lane's two columns
  int colv[2];
  bool colok[2];
  float cs[2], cs2k[2], bv[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const int c = 32 * wave + 16 * hf + (lane & 15);
    colv[hf] = c;
    colok[hf] = c < Nc;
    const int cc = colok[hf] ? c : 0;
    cs[hf] = colok[hf] ? colscale[cc] : 0.f;  // 2^(e_n - 11 - ap_exp)
    cs2k[hf] = cs[hf] * 2048.0f;
    bv[hf] = ((EPI & WS_BIAS) != 0 && colok[hf]) ? a.bias[cc] : 0.f;
  }
  float* const pl = reinterpret_cast<float*>(smem + PL0);
  if constexpr (PROJ) {  // P in LDS (the epilogue reads a lane's 2 columns per tile: 8 VGPRs fewer)
    for (int i = tid; i < MAXPROJ * BN; i += 256) {
      const int q = i / BN, cc = i % BN;
      pl[i] = (q < a.nproj && cc < Nc) ? a.proj[(int64_t)q * Nc + cc] : 0.f;
    }
  }
  const int64_t ldc = a.ldc;
  const __amdgpu_buffer_rsrc_t crsrc =
      __builtin_amdgcn_make_buffer_rsrc(a.c, 0, a.c ? (int)(M * ldc * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t zrsrc =
      __builtin_amdgcn_make_buffer_rsrc(a.z, 0, PROJ ? (int)(M * a.ldz * 4) : 0, 0x00020000);

  // ---- the LDS-DMA of one tile (rows clamped into the image: tail rows repeat row M - 1, their
  //      stores are dropped by the buffer range / row check)
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  auto glds16 = [](const uint16_t* src, uint32_t dst) {  // dst is wave-uniform: an SGPR for M0
    unsigned keep;
    const uint32_t d = __builtin_amdgcn_readfirstlane(dst);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(d) : "memory");
  };
  const int drow = lane >> 2;
  const int dkq = (lane & 3) ^ ((drow >> 2) & 3);  // the k-quarter this lane's 16 B slot holds
  auto dma = [&](int tt, int buf) {
    const int tc = min(tt, ntiles - 1);
    const int64_t row = min((int64_t)tc * H2R_ROWS + drow, M - 1);
    const uint16_t* rp = a.ap + row * ld;
#pragma unroll
    for (int i = 0; i < QW; ++i) {
      const int b = wave + 4 * i;
      if (b < NBLK) {
        const int p = b / NK, s = b - p * NK;
        const int k = 32 * s + 8 * dkq;
        glds16(rp + p * a.ap_ps + (k < ld ? k : 0), lds0 + (uint32_t)(buf * ABUF + b * KB));
      } else {
        glds16(rp, lds0 + (uint32_t)SCR);
      }
    }
  };
  auto wait_vm = [](auto nc) {  // vmcnt(N) alone (expcnt / lgkmcnt at their maxima), gfx9 encoding
    constexpr int N = decltype(nc)::value;
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  };
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t foff = (uint32_t)(fr * 64 + 16 * (fq ^ ((fr >> 2) & 3)));

  // z of tile tp: the 4 column blocks' partials in order; wave w stores rows 4w .. +4 (one store)
  auto zfinal = [&](int tp, int zb) {
    const float* zp = reinterpret_cast<const float*>(smem + ZP0 + zb * ZPB);
    const int r = 4 * wave + ((lane >> 2) & 3), q = lane & 3;
    float zv = 0.f;
    if constexpr (PROJ) {
      const int i = r * MAXPROJ + q;
      zv = ((zp[i] + zp[64 + i]) + zp[128 + i]) + zp[192 + i];
    }
    const int64_t row = (int64_t)tp * H2R_ROWS + r;
    const uint32_t zoff = (PROJ && lane < 16 && q < a.nproj && tp >= 0 && row < M) ? (uint32_t)((row * a.ldz + q) * 4)
                                                                                    : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(zv), zrsrc, (int)zoff, 0, 0);
  };

  wait_vm(std::integral_constant<int, 0>{});  // B / constants landed before the ring's counted waits
  if constexpr (!(LAB & 4)) {
    dma(t, 0);
    dma(t + G, 1);
  }
  int tp = -1;
  for (int it = 0;; ++it) {
    // DMA(it) landed: issued after it were DMA(it + 1) and every store since (see S)
    if constexpr (!(LAB & 4)) {
      if (it == 0) wait_vm(std::integral_constant<int, QW>{});
      else if (it == 1) wait_vm(std::integral_constant<int, QW + S>{});
      else wait_vm(std::integral_constant<int, QW + S + 8>{});
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous tile's projection partials
    __builtin_amdgcn_s_barrier();
    zfinal(tp, (it + 1) & 1);
    if constexpr (!(LAB & 4)) dma(t + 2 * G, (it + 2) % NBUF);
    const char* cur = smem + (it % NBUF) * ABUF;
    floatx4 x0, x1, h0, h1;
    if (active && !(LAB & 1)) {
      // A fragments one k-step ahead (the reads of step s + 1 in flight under step s's 6 MFMAs)
      f16x8 ah[2], al[2];
      ah[0] = *reinterpret_cast<const f16x8*>(cur + foff);
      al[0] = *reinterpret_cast<const f16x8*>(cur + NK * KB + foff);
      static_for<NK>([&](auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        constexpr int u = s & 1;
        if constexpr (s + 1 < NK) {
          ah[u ^ 1] = *reinterpret_cast<const f16x8*>(cur + (s + 1) * KB + foff);
          al[u ^ 1] = *reinterpret_cast<const f16x8*>(cur + (NK + s + 1) * KB + foff);
        }
        if constexpr ((LAB & 8) != 0) __builtin_amdgcn_sched_barrier(0);  // lab: force the prefetch order
        h2r_mfma<s == 0>(x0, ah[u], bl[s][0]);
        h2r_mfma<s == 0>(x1, ah[u], bl[s][1]);
        h2r_mfma<s == 0>(h0, ah[u], bh[s][0]);
        h2r_mfma<s == 0>(h1, ah[u], bh[s][1]);
        h2r_mfma<false>(x0, al[u], bh[s][0]);
        h2r_mfma<false>(x1, al[u], bh[s][1]);
        if constexpr ((LAB & 8) != 0) __builtin_amdgcn_sched_barrier(0);
      });
      h2r_mfma_end(x0, x1, h0, h1);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) x0[r] = x1[r] = h0[r] = h1[r] = 0.f;
      if constexpr ((LAB & 1) != 0) x0[0] = (float)(*reinterpret_cast<const f16x8*>(cur + foff))[0];
    }
    // ---- epilogue of tile t
    float zpq[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) zpq[j] = 0.f;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const floatx4& xx = hf ? x1 : x0;
      const floatx4& hh = hf ? h1 : h0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = 4 * (lane >> 4) + i;
        const int64_t row = (int64_t)t * H2R_ROWS + rl;
        float v = fmaf(hh[i], cs2k[hf], xx[i] * cs[hf]) + bv[hf];
        if constexpr ((EPI & WS_RELU) != 0) v = fmaxf(v, 0.f);
        if constexpr ((EPI & WS_DROP) != 0)  // == keep_elem(seed, row·Nc + col, thresh), bit for bit
          v = keep_elem(seed, (uint32_t)row * (uint32_t)Nc + (uint32_t)colv[hf], a.keep_thresh) ? v * a.drop_scale : 0.f;
        if (!colok[hf]) v = 0.f;
        if constexpr (!(LAB & 2)) {
          const uint32_t off = (colok[hf] && row < M) ? (uint32_t)((row * ldc + colv[hf]) * 4) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), crsrc, (int)off, 0, 0);
        }
        if constexpr (PROJ) {
#pragma unroll
          for (int q = 0; q < MAXPROJ; ++q) zpq[4 * i + q] = fmaf(v, pl[q * BN + colv[hf]], zpq[4 * i + q]);
        }
      }
    }
    if constexpr (PROJ) {
      // reduce-and-split over the 16 lanes of the row group: lane l ends with index (l & 15) = 4 i + q
      float z8[8], z4[4], z2[2];
      const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
#pragma unroll
      for (int j = 0; j < 8; ++j) z8[j] = (b3 ? zpq[j + 8] : zpq[j]) + __shfl_xor(b3 ? zpq[j] : zpq[j + 8], 8);
#pragma unroll
      for (int j = 0; j < 4; ++j) z4[j] = (b2 ? z8[j + 4] : z8[j]) + __shfl_xor(b2 ? z8[j] : z8[j + 4], 4);
#pragma unroll
      for (int j = 0; j < 2; ++j) z2[j] = (b1 ? z4[j + 2] : z4[j]) + __shfl_xor(b1 ? z4[j] : z4[j + 2], 2);
      const float z1 = (b0 ? z2[1] : z2[0]) + __shfl_xor(b0 ? z2[0] : z2[1], 1);
      // lane l: row 4 (l >> 4) + ((l >> 2) & 3), q = l & 3
      float* zp = reinterpret_cast<float*>(smem + ZP0 + (it & 1) * ZPB);
      zp[wave * 64 + (4 * (lane >> 4) + ((lane >> 2) & 3)) * MAXPROJ + (lane & 3)] = z1;
    }
    if constexpr ((LAB & 2) != 0) {  // keep the C stores' count for the vmcnt accounting
#pragma unroll
      for (int j = 0; j < 8; ++j)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x0[j & 3] + h1[j & 3]), crsrc, (int)0x80000000u, 0, 0);
    }
    tp = t;
    t += G;
    if (t >= ntiles) {
      wait_vm(std::integral_constant<int, 0>{});  // no DMA may outlive the block's LDS
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      zfinal(tp, it & 1);
      break;
    }
  }
}

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

// reference stream: read A (uint4) and write C (float4), 1 block per CU sweep
__global__ __launch_bounds__(256) void stream_kernel(const uint4* __restrict__ a, int64_t na, float4* __restrict__ c,
                                                     int64_t nc) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
  uint32_t acc = 0;
  for (int64_t i = i0; i < na; i += st) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.w;
  }
  for (int64_t i = i0; i < nc; i += st) c[i] = make_float4((float)acc, 0.f, 0.f, 0.f);
}

constexpr int EPIF = WS_BIAS | WS_RELU | WS_DROP | WS_PROJ;
static NTArgs g_n;
static uint4* g_b;
static float* g_cs;
static int g_nt32, g_nt16;
template <int LAB>
void old32() { gemm_nt_h2_kernel<21, EPIF, LAB><<<256, 256>>>(g_n, g_b, g_cs, g_nt32); }
template <int LAB, int E = EPIF>
void ring16() { gemm_nt_h2r_kernel<11, E, LAB><<<512, 256>>>(g_n, g_b, g_cs, g_nt16); }
static const uint4* g_sa;
static float4* g_sc;
static int64_t g_M = 203769;
void stream() { stream_kernel<<<1024, 256>>>(g_sa, g_M * 336 * 2 * 2 / 16, g_sc, g_M * 128 / 4); }

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 9;
  const int64_t M = argc > 2 ? std::atoll(argv[2]) : 203769, F = 166, LD = 336, NR = 128;  // M: shard sizes too
  std::vector<float> hx(M * LD, 0.f);
  {
    std::mt19937 g(1);
    std::normal_distribution<float> d(0.f, 1.f);
    for (int64_t r = 0; r < M; ++r)
      for (int c = 0; c < F; ++c) {
        hx[r * LD + c] = d(g) * 0.7f;
        hx[r * LD + 168 + c] = d(g);
      }
  }
  float* xa;
  CK(hipMalloc(&xa, M * LD * 4));
  CK(hipMemcpy(xa, hx.data(), M * LD * 4, hipMemcpyHostToDevice));
  uint16_t* imh;
  CK(hipMalloc(&imh, 2 * M * LD * 2));
  gnn_split_h2_f32(xa, LD, M, LD, imh, LD, M * LD, 0, LD, 11, nullptr);  // the image holds x·2^11
  std::vector<float> hw1(NR * F), hw2(NR * F), hb(NR), hp(4 * NR);
  {
    std::mt19937 g(5);
    std::normal_distribution<float> d(0.f, 1.f);
    for (auto& v : hw1) v = d(g) * 0.08f;
    for (auto& v : hw2) v = d(g) * 0.08f;
    for (auto& v : hb) v = d(g) * 0.1f;
    for (auto& v : hp) v = d(g);
  }
  auto up = [](const std::vector<float>& h) {
    float* p;
    CK(hipMalloc(&p, h.size() * 4));
    CK(hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return p;
  };
  float *w1 = up(hw1), *w2 = up(hw2), *bias = up(hb), *proj = up(hp);
  float *c, *z;
  CK(hipMalloc(&c, M * NR * 4));
  CK(hipMalloc(&z, M * 4 * 4));
  NTArgs n{};
  n.M = M; n.Nc = NR; n.k1 = F; n.k2 = F; n.w1 = w1; n.w2 = w2; n.ldw1 = F; n.ldw2 = F; n.c = c; n.ldc = NR;
  n.bias = bias; n.relu = 1; n.dropout = 1; n.keep_thresh = (uint32_t)(0.5 * 16777216.0); n.drop_scale = 2.f;
  n.seed = 1234; n.proj = proj; n.nproj = 4; n.z = z; n.ldz = 4;
  n.ap = imh; n.ap_ld = LD; n.ap_col2 = 168; n.ap_ps = M * LD; n.ap_h2 = 1; n.ap_exp = 11;
  CK(hipMalloc(&g_b, 21 * 3 * 256 * 16 + 128 * 4));
  g_cs = reinterpret_cast<float*>(g_b + 21 * 3 * 256);
  g_n = n;
  ws_prep_h2_kernel<<<WS_PREP_GRID, WS_PREP_THREADS>>>(h2_prep_of(g_n, g_b));
  g_M = M;
  g_nt32 = (int)ceil_div(M, 32);
  g_nt16 = (int)ceil_div(M, 16);
  g_sa = reinterpret_cast<const uint4*>(imh);
  CK(hipMalloc(&g_sc, M * NR * 4));
  {  // the two forms agree (same masks, f32 rounding)
    std::vector<float> r0(M * NR), r1(M * NR);
    old32<0>();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r0.data(), c, M * NR * 4, hipMemcpyDeviceToHost));
    ring16<0>();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r1.data(), c, M * NR * 4, hipMemcpyDeviceToHost));
    double e = 0, nn = 0;
    size_t zd = 0;
    for (size_t i = 0; i < r0.size(); ++i) {
      e += (double)(r0[i] - r1[i]) * (r0[i] - r1[i]);
      nn += (double)r0[i] * r0[i];
      zd += (r0[i] == 0.f) != (r1[i] == 0.f);
    }
    std::printf("32-row vs 16-row ring: relL2 %.3g, zero patterns differing %zu of %zu\n", std::sqrt(e / nn), zd, r0.size());
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V { const char* name; void (*f)(); std::vector<float> t; };
  std::vector<V> vs = {
      {"stream A + C (1024 blocks)", stream, {}},
      {"NT 32-row", old32<0>, {}}, {"NT 32-row no MFMA", old32<1>, {}},
      {"NT ring16", ring16<0>, {}}, {"NT ring16 prefetch pinned", ring16<8>, {}},
      {"NT ring16 prefetch pinned MFMA only", ring16<8 | 2 | 4>, {}}, {"NT ring16 no MFMA", ring16<1>, {}}, {"NT ring16 no epilogue", ring16<2>, {}},
      {"NT ring16 no DMA", ring16<4>, {}}, {"NT ring16 MFMA only", ring16<2 | 4>, {}},
      {"NT ring16 DMA only", ring16<1 | 2>, {}}, {"NT ring16 epilogue only", ring16<1 | 4>, {}},
      {"NT ring16 no dropout", ring16<0, WS_BIAS | WS_RELU | WS_PROJ>, {}},
      {"NT ring16 no proj", ring16<0, WS_BIAS | WS_RELU | WS_DROP>, {}}};
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      v.f();
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) v.f();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms * 1000.f / 5);
    }
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    std::printf("%-30s %8.1f us (min %.1f)\n", v.name, v.t[v.t.size() / 2], v.t[0]);
  }
  return 0;
}
