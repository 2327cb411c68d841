// Shared helpers for libgnnmp (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <type_traits>
#include <utility>

#include "../../include/gnnmp.h"

namespace gnnmp {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

void set_last_error(const std::string& msg);

inline gnn_status fail(gnn_status s, const char* fn, const char* what) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s", fn, what);
  set_last_error(buf);
  return s;
}

inline gnn_status hip_check(hipError_t e, const char* fn) {
  if (e == hipSuccess) return GNN_OK;
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: HIP error %d (%s)", fn, static_cast<int>(e),
                hipGetErrorString(e));
  set_last_error(buf);
  return GNN_ERR_HIP;
}

#define GNN_HIP_TRY(expr)                                 \
  do {                                                    \
    gnn_status _s = ::gnnmp::hip_check((expr), __func__); \
    if (_s != GNN_OK) return _s;                          \
  } while (0)

#define GNN_LAUNCH_CHECK() GNN_HIP_TRY(hipGetLastError())

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace (256-B aligned carves).
struct WorkspaceCarver {
  char* base;
  size_t cap;
  size_t used = 0;
  bool ok = true;
  WorkspaceCarver(void* p, size_t c) : base(static_cast<char*>(p)), cap(c) {}
  template <typename T>
  T* take(size_t count) {
    size_t off = align_up(used, 256);
    size_t bytes = align_up(count * sizeof(T), 256);
    if (off + bytes > cap) {
      ok = false;
      return nullptr;
    }
    used = off + bytes;
    return reinterpret_cast<T*>(base + off);
  }
};

// Sizes-only twin of WorkspaceCarver (same carve rules).
struct WorkspaceSizer {
  size_t used = 0;
  template <typename T>
  void take(size_t count) {
    used = align_up(used, 256) + align_up(count * sizeof(T), 256);
  }
};

}  // namespace gnnmp
