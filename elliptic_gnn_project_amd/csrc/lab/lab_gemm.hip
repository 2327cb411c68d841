// Kernel lab (not part of the library): timing ablations of the split-image GEMMs on the SAGE
// layer-1 shape (M = 203,769 rows, image [3][M][336], 128 columns): the TN (dz form + mask) and
// the NT (bias + ReLU + dropout + projection), variants interleaved in one process, median of
// rounds.  Built by `make lab` (csrc/Makefile); run on the GPU box:  ./lab_gemm [rounds]
#define GNNMP_LAB 1
#include "../gemm_planes.hip"
#include "../gemm_ws.hip"

#include <algorithm>
#include <cstring>
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
void nt(const TNArgs&, const NTArgs& a, const uint4* img, int, int ntiles) {
  gemm_nt_planes_kernel<WS_BIAS | WS_RELU | WS_DROP | WS_PROJ, LAB><<<256, 256>>>(a, img, ntiles);
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
  struct V { const char* name; void (*f)(const TNArgs&, const NTArgs&, const uint4*, int, int); std::vector<float> t; };
  std::vector<V> vs = {
      {"TN production", tn<0>, {}}, {"TN no MFMA", tn<1>, {}}, {"TN no staging", tn<2>, {}},
      {"TN no frag reads", tn<4>, {}}, {"TN no barrier", tn<8>, {}}, {"TN MFMA+frags", tn<2 | 8>, {}},
      {"TN MFMA only", tn<2 | 4 | 8>, {}}, {"TN staging only", tn<1 | 4>, {}},
      {"NT production", nt<0>, {}}, {"NT no MFMA", nt<1>, {}}, {"NT no epilogue", nt<2>, {}},
      {"NT no staging", nt<4>, {}}, {"NT no mid barrier", nt<8>, {}}, {"NT MFMA+frags only", nt<2 | 4 | 8>, {}},
      {"NT epilogue only", nt<1 | 4>, {}}};
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
