// Kernel lab (not part of the library): the half-pair NT (gemm_nt_h2_kernel: f16 hi / lo planes,
// 3 products per k-step) against the split-bf16 image NT (6 products) on the SAGE layer-1 shape
// (M = 203,769, [agg | x] = 166 + 166 padded to 168 each, N = 128, bias + ReLU + dropout +
// projection).  Accuracy of both against a float64 host reference on sampled rows, then timings
// (variants interleaved, median).   make -C elliptic_gnn_project_amd/csrc labh2
#define GNNMP_LAB 1
#include "../gemm_planes.hip"
#include "../gemm_ws.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
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

using namespace gnnmp;

__global__ void split_h2_kernel(const float* x, int64_t n2, uint16_t* img, int64_t ps) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n2) return;
  uint32_t h, l;
  split_h2_pair(x[2 * i], x[2 * i + 1], h, l);
  reinterpret_cast<uint32_t*>(img)[i] = h;
  reinterpret_cast<uint32_t*>(img + ps)[i] = l;
}

constexpr int EPIF = WS_BIAS | WS_RELU | WS_DROP | WS_PROJ;
constexpr int EPIN = WS_BIAS | WS_RELU | WS_PROJ;
static NTArgs g_h;
static uint4* g_bh;
static float* g_cs;
template <int LAB, int E = EPIF>
void ntp(const NTArgs& a, const uint4* img, int ntiles) {
  gemm_nt_planes_kernel<21, E, LAB><<<256, 256>>>(a, img, ntiles);
}
template <int LAB, int E = EPIF>
void nth(const NTArgs&, const uint4*, int ntiles) {
  gemm_nt_h2_kernel<21, E, LAB><<<256, 256>>>(g_h, g_bh, g_cs, ntiles);
}

static TNArgs g_tp, g_th;
template <int LAB>
void tnp(const NTArgs&, const uint4*, int) {
  gemm_tn_planes_kernel<true, true, 11, false, LAB><<<256, 256>>>(g_tp);
}
template <int LAB>
void tnh(const NTArgs&, const uint4*, int) {
  gemm_tn_h2_kernel<11, false, LAB><<<256, 256>>>(g_th);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 9;
  const int64_t M = 203769, F = 166, LD = 336, NR = 128;
  std::vector<float> hx(M * LD, 0.f);
  {
    std::mt19937 g(1);
    std::normal_distribution<float> d(0.f, 1.f);
    for (int64_t r = 0; r < M; ++r)
      for (int c = 0; c < F; ++c) {
        hx[r * LD + c] = d(g) * 0.7f;  // agg: a mean, slightly narrower
        hx[r * LD + 168 + c] = d(g);
      }
  }
  float* xa;
  CK(hipMalloc(&xa, M * LD * 4));
  CK(hipMemcpy(xa, hx.data(), M * LD * 4, hipMemcpyHostToDevice));
  uint16_t *img, *imh;
  CK(hipMalloc(&img, 3 * M * LD * 2));
  CK(hipMalloc(&imh, 2 * M * LD * 2));
  gnn_split_planes_f32(xa, LD, M, LD, img, LD, M * LD, 0, LD, nullptr);
  split_h2_kernel<<<(unsigned)ceil_div(M * LD / 2, 256), 256>>>(xa, M * LD / 2, imh, M * LD);
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
  float *c, *z, *c2, *z2;
  CK(hipMalloc(&c, M * NR * 4));
  CK(hipMalloc(&z, M * 4 * 4));
  CK(hipMalloc(&c2, M * NR * 4));
  CK(hipMalloc(&z2, M * 4 * 4));
  NTArgs n{};
  n.M = M; n.Nc = NR; n.k1 = F; n.k2 = F; n.w1 = w1; n.w2 = w2; n.ldw1 = F; n.ldw2 = F; n.c = c; n.ldc = NR;
  n.bias = bias; n.relu = 1; n.dropout = 1; n.keep_thresh = (uint32_t)(0.5 * 16777216.0); n.drop_scale = 2.f;
  n.seed = 1234; n.proj = proj; n.nproj = 4; n.z = z; n.ldz = 4;
  n.ap = img; n.ap_ld = LD; n.ap_col2 = 168; n.ap_ps = M * LD;
  uint4* bimg;
  CK(hipMalloc(&bimg, 21 * 3 * 256 * 16));
  ws_prep_kernel<<<21, 256>>>(n, bimg, 21, nullptr, 0, 168);
  CK(hipMalloc(&g_bh, 21 * 3 * 256 * 16));
  CK(hipMalloc(&g_cs, 128 * 4));
  g_h = n; g_h.ap = imh; g_h.c = c2; g_h.z = z2;
  ws_prep_h2_kernel<<<21, 256>>>(g_h, g_bh, g_cs, 168);
  const int ntiles = (int)ceil_div(M, 32);

  // accuracy: no dropout (deterministic), C vs float64 on sampled rows
  {
    NTArgs a = n; a.dropout = 0;
    NTArgs b = g_h; b.dropout = 0;
    gemm_nt_planes_kernel<21, EPIN, 0><<<256, 256>>>(a, bimg, ntiles);
    gemm_nt_h2_kernel<21, EPIN, 0><<<256, 256>>>(b, g_bh, g_cs, ntiles);
    CK(hipDeviceSynchronize());
    std::vector<float> r0(M * NR), r1(M * NR), q0(M * 4), q1(M * 4);
    CK(hipMemcpy(r0.data(), c, M * NR * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r1.data(), c2, M * NR * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q0.data(), z, M * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q1.data(), z2, M * 16, hipMemcpyDeviceToHost));
    double e0 = 0, e1 = 0, nrm = 0, m0 = 0, m1 = 0, ze0 = 0, ze1 = 0, zn = 0;
    for (int64_t r = 0; r < M; r += 97) {
      std::vector<double> hrow(NR);
      for (int j = 0; j < NR; ++j) {
        double s = hb[j];
        for (int k = 0; k < F; ++k) s += (double)hx[r * LD + k] * hw1[j * F + k] + (double)hx[r * LD + 168 + k] * hw2[j * F + k];
        s = std::max(s, 0.0);
        hrow[j] = s;
        const double d0 = r0[r * NR + j] - s, d1 = r1[r * NR + j] - s;
        e0 += d0 * d0; e1 += d1 * d1; nrm += s * s;
        m0 = std::max(m0, std::fabs(d0)); m1 = std::max(m1, std::fabs(d1));
      }
      for (int q = 0; q < 4; ++q) {
        double zz = 0;
        for (int j = 0; j < NR; ++j) zz += hrow[j] * hp[q * NR + j];
        ze0 += (q0[r * 4 + q] - zz) * (q0[r * 4 + q] - zz);
        ze1 += (q1[r * 4 + q] - zz) * (q1[r * 4 + q] - zz);
        zn += zz * zz;
      }
    }
    std::printf("accuracy vs f64 (every 97th row): split-bf16 relL2 %.3g (max abs %.3g) z %.3g | half-pair relL2 %.3g (max abs %.3g) z %.3g\n",
                std::sqrt(e0 / nrm), m0, std::sqrt(ze0 / zn), std::sqrt(e1 / nrm), m1, std::sqrt(ze1 / zn));
    // dropout masks agree: zero patterns of C with dropout on
    nth<0>(n, bimg, ntiles);
    ntp<0>(n, bimg, ntiles);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r0.data(), c, M * NR * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r1.data(), c2, M * NR * 4, hipMemcpyDeviceToHost));
    size_t zd = 0;
    for (size_t i = 0; i < r0.size(); ++i) zd += (r0[i] == 0.f) != (r1[i] == 0.f);
    std::printf("dropout: %zu of %zu zero patterns differ (ReLU ties aside)\n", zd, r0.size());
  }
  // ---- TN: dW = Gᵀ·[agg | x], G = (dz·P) ⊙ [h > 0] · 2 (the SAGE hidden layer's weight gradient)
  std::vector<float> hh(M * NR), hdz(M * 4);
  {
    std::mt19937 g(2);
    std::normal_distribution<float> d(0.f, 1.f);
    for (auto& v : hh) v = d(g);
    for (auto& v : hdz) v = d(g) * 1e-5f;  // loss gradients / n_train: small
  }
  float *dh = up(hh), *ddz = up(hdz);
  const int nblk = 256;
  const int64_t stride = (NR * 332 + NR + 4 * NR + 4 + 63) / 64 * 64;
  float* slab;
  CK(hipMalloc(&slab, nblk * stride * 4));
  TNArgs ta{};
  ta.M = M; ta.Nr = NR; ta.dz = ddz; ta.lddz = 4; ta.proj = proj; ta.nproj = 4; ta.h = dh; ta.ldh = NR; ta.hscale = 2.f;
  ta.k1 = F; ta.k2 = F; ta.slab = slab; ta.slab_stride = stride;
  ta.rows_per_block = ceil_div(ceil_div(M, 32), nblk) * 32;
  ta.ap = img; ta.ap_ld = LD; ta.ap_col2 = 168; ta.ap_ps = M * LD;
  g_tp = ta;
  g_th = ta; g_th.ap = imh;
  {
    const int64_t Ms = 20000;  // accuracy on a prefix of the rows (f64 host reference)
    TNArgs pa = g_tp, ha = g_th;
    pa.M = ha.M = Ms;
    pa.rows_per_block = ha.rows_per_block = ceil_div(ceil_div(Ms, 32), nblk) * 32;
    std::vector<double> ref(NR * 332, 0.0);
    for (int64_t m = 0; m < Ms; ++m)
      for (int n2 = 0; n2 < NR; ++n2) {
        if (hh[m * NR + n2] <= 0.f) continue;
        double gg = 0;
        for (int q = 0; q < 4; ++q) gg += (double)hdz[m * 4 + q] * hp[q * NR + n2];
        gg *= 2.0;
        for (int k = 0; k < F; ++k) {  // slab layout: dW1 [Nr][k1], then dW2 [Nr][k2]
          ref[n2 * F + k] += gg * hx[m * LD + k];
          ref[NR * F + n2 * F + k] += gg * hx[m * LD + 168 + k];
        }
      }
    auto run = [&](const char* name, bool h2) {
      CK(hipMemset(slab, 0, nblk * stride * 4));
      if (h2) gemm_tn_h2_kernel<11, false, 0><<<nblk, 256>>>(ha);
      else gemm_tn_planes_kernel<true, true, 11, false, 0><<<nblk, 256>>>(pa);
      CK(hipDeviceSynchronize());
      std::vector<float> hs(nblk * stride);
      CK(hipMemcpy(hs.data(), slab, hs.size() * 4, hipMemcpyDeviceToHost));
      double e = 0, nn = 0;
      for (int i = 0; i < NR * 332; ++i) {
        double v = 0;
        for (int b = 0; b < nblk; ++b) v += hs[b * stride + i];
        e += (v - ref[i]) * (v - ref[i]);
        nn += ref[i] * ref[i];
      }
      std::printf("TN %s: dW relL2 vs f64 %.3g\n", name, std::sqrt(e / nn));
    };
    run("split-bf16 planes", false);
    run("half-pair", true);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V { const char* name; void (*f)(const NTArgs&, const uint4*, int); std::vector<float> t; };
  std::vector<V> vs = {
      {"NT planes (bf16 x6)", ntp<0>, {}}, {"NT planes no epi", ntp<2>, {}}, {"NT planes no staging", ntp<4>, {}},
      {"NT planes MFMA only", ntp<2 | 4 | 8>, {}},
      {"NT half-pair", nth<0>, {}}, {"NT half-pair no epi", nth<2>, {}}, {"NT half-pair no staging", nth<4>, {}},
      {"NT half-pair MFMA only", nth<2 | 4>, {}}, {"NT half-pair no MFMA", nth<1>, {}},
      {"NT half-pair no dropout", nth<0, EPIN>, {}},
      {"TN planes (bf16 x6)", tnp<0>, {}}, {"TN planes MFMA only", tnp<2 | 8>, {}},
      {"TN half-pair", tnh<0>, {}}, {"TN half-pair no staging", tnh<2>, {}}, {"TN half-pair no MFMA", tnh<1>, {}}};
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      v.f(n, bimg, ntiles);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) v.f(n, bimg, ntiles);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms * 1000.f / 5);
    }
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    std::printf("%-28s %8.1f us (min %.1f)\n", v.name, v.t[v.t.size() / 2], v.t[0]);
  }
  return 0;
}
