// Kernel lab: times libgnnmp kernels through the C ABI on the Elliptic SAGE-preset shapes
// (hipEvent timing, all variants interleaved in one process, median of rounds).
//   ./bench_gemm [M] [rounds]
// Not part of the library; built by `make lab`.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <cmath>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../include/gnnmp.h"

extern "C" gnn_status gnnx_gemm_nt_variant_f32(const gnn_gemm_nt_params* p, int variant, gnn_stream_t stream);

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)
#define GK(x)                                                                  \
  do {                                                                         \
    gnn_status s = (x);                                                        \
    if (s != GNN_OK) {                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, gnn_status_string(s), gnn_last_error()); \
      std::exit(1);                                                            \
    }                                                                          \
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

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  template <typename F>
  float run(F f, int reps) {
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
  }
};

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? std::atoll(argv[1]) : 203769;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 7;
  const int64_t F = std::getenv("LAB_F") ? std::atoll(std::getenv("LAB_F")) : 166, H = 128;
  float* agg = dev_rand(M * F, 1.f, 1);
  float* x = dev_rand(M * F, 1.f, 2);
  float* bt = dev_rand(2 * F * H, 0.08f, 3);
  float* bias = dev_rand(H, 0.1f, 4);
  float* proj = dev_rand(4 * H, 0.1f, 5);
  float *c, *z;
  CK(hipMalloc(&c, M * H * sizeof(float)));
  CK(hipMalloc(&z, M * 4 * sizeof(float)));
  float* dz = dev_rand(M * 4, 1e-3f, 6);

  gnn_gemm_nt_params p{};
  p.M = M; p.N = H;
  p.a1 = agg; p.lda1 = F; p.k1 = F;
  p.a2 = x; p.lda2 = F; p.k2 = F;
  p.bt = bt; p.ldb = H;
  p.c = c; p.ldc = H; p.bias = bias; p.relu = 1; p.dropout_p = 0.5f; p.seed = 1234;
  p.proj = proj; p.nproj = 4; p.z = z; p.ldz = 4;
  gnn_gemm_nt_params plain = p;
  plain.bias = nullptr; plain.relu = 0; plain.dropout_p = 0.f; plain.proj = nullptr; plain.nproj = 0; plain.z = nullptr;

  const double flops = 2.0 * M * (2 * F) * H;
  Timer T;
  const int nvar = 7;
  std::vector<std::vector<float>> t_epi(nvar), t_plain(nvar);
  // correctness: every variant must agree bitwise with variant 0 (same k-ordered fmaf chain)
  std::vector<float> ref(M * H), got(M * H);
  GK(gnnx_gemm_nt_variant_f32(&p, 0, nullptr));
  CK(hipMemcpy(ref.data(), c, M * H * 4, hipMemcpyDeviceToHost));
  for (int v = 1; v < nvar; ++v) {
    if (v >= 4) continue;  // ablations: outputs are meaningless  // ablations: outputs are meaningless
    GK(gnnx_gemm_nt_variant_f32(&p, v, nullptr));
    CK(hipMemcpy(got.data(), c, M * H * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    double maxd = 0.0;
    for (size_t i = 0; i < got.size(); ++i) {
      bad += got[i] != ref[i];
      double d = std::fabs((double)got[i] - (double)ref[i]) / (1e-3 + std::fabs((double)ref[i]));
      maxd = d > maxd ? d : maxd;
    }
    std::printf("variant %d mismatches vs 0: %zu  max rel diff %.2e\n", v, bad, maxd);
  }
  // LAB_ONLY=v[,wform]: time one variant only (for rocprofv3 --pmc passes); no other sections
  if (const char* only = std::getenv("LAB_ONLY")) {
    const int v = std::atoi(only);
    gnn_gemm_nt_params q = p;
    if (std::strchr(only, 'w')) {
      float* w = dev_rand(2 * F * H, 0.08f, 7);
      q.bt = nullptr; q.w1 = w; q.w2 = w + F * H; q.ldw1 = F; q.ldw2 = F;
    }
    for (int r = 0; r < rounds; ++r) GK(gnnx_gemm_nt_variant_f32(&q, v, nullptr));
    CK(hipDeviceSynchronize());
    std::printf("LAB_ONLY %s done\n", only);
    return 0;
  }
  for (int r = 0; r < rounds; ++r) {
    for (int v = 0; v < nvar; ++v) {
      t_epi[v].push_back(T.run([&] { gnnx_gemm_nt_variant_f32(&p, v, nullptr); }, 5));
      t_plain[v].push_back(T.run([&] { gnnx_gemm_nt_variant_f32(&plain, v, nullptr); }, 5));
    }
  }
  auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  for (int v = 0; v < nvar; ++v) {
    float a = med(t_epi[v]), b = med(t_plain[v]);
    std::printf("NT variant %d: fused-epilogue %8.1f us (%6.1f TF)   plain %8.1f us (%6.1f TF)\n", v, a,
                flops / a * 1e-6, b, flops / b * 1e-6);
  }
  // B read in place from Linear weights W1/W2 [H, F] (the production forward form)
  {
    float* w = dev_rand(2 * F * H, 0.08f, 7);
    gnn_gemm_nt_params pw = p;
    pw.bt = nullptr; pw.w1 = w; pw.w2 = w + F * H; pw.ldw1 = F; pw.ldw2 = F;
    for (int v : {0, 1, 2, 3}) {
      std::vector<float> tw;
      for (int r = 0; r < rounds; ++r) tw.push_back(T.run([&] { gnnx_gemm_nt_variant_f32(&pw, v, nullptr); }, 5));
      float a = med(tw);
      std::printf("NT variant %d w1/w2 form: fused-epilogue %8.1f us (%6.1f TF)\n", v, a, flops / a * 1e-6);
    }
  }
  // TN (dz form + mask), the backward weight-gradient shape
  gnn_gemm_tn_params q{};
  q.M = M; q.Nr = H; q.dz = dz; q.lddz = 4; q.proj = proj; q.nproj = 4; q.h = c; q.ldh = H; q.hscale = 2.f;
  q.a1 = agg; q.lda1 = F; q.k1 = F; q.a2 = x; q.lda2 = F; q.k2 = F;
  size_t wsb = 0;
  GK(gnn_gemm_tn_workspace_size(M, H, 2 * F, 4, &wsb));
  void* ws;
  CK(hipMalloc(&ws, wsb));
  float* out;
  CK(hipMalloc(&out, (H * 2 * F + H + 4 * H + 4) * sizeof(float)));
  std::vector<float> tt;
  for (int r = 0; r < rounds; ++r) tt.push_back(T.run([&] { gnn_gemm_tn_f32(&q, out, ws, wsb, nullptr); }, 5));
  float a = med(tt);
  std::printf("TN dz+mask: %8.1f us (%6.1f TF)\n", a, flops / a * 1e-6);
  return 0;
}
