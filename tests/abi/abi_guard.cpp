// The ABI contract of include/omega.h -- no C++ exception and no abort crosses the boundary -- checked
// through public entry points on the CPU (tests/test_capi.py::test_abi_guard_maps_host_allocation_failure).
// This program replaces the global operator new (the library's allocations resolve to it) with one that
// throws std::bad_alloc while armed, then calls entry points that allocate host memory: each must return
// OMEGA_ENOMEM with a message instead of terminating the process.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/omega.h"

static bool g_armed = false;

void* operator new(std::size_t n) {
  if (g_armed) throw std::bad_alloc();
  if (void* p = std::malloc(n ? n : 1)) return p;
  throw std::bad_alloc();
}
void* operator new[](std::size_t n) { return operator new(n); }
void operator delete(void* p) noexcept { std::free(p); }
void operator delete[](void* p) noexcept { std::free(p); }
void operator delete(void* p, std::size_t) noexcept { std::free(p); }
void operator delete[](void* p, std::size_t) noexcept { std::free(p); }

static int check(const char* what, int rc, int want) {
  std::printf("%s: %d (want %d)\n", what, rc, want);
  return rc == want ? 0 : 1;
}

int main() {
  int bad = 0;
  omega_config cfg;
  omega_config_default(&cfg);
  // 1) the context itself cannot be allocated: ENOMEM, no context handed out
  omega_ctx* c = nullptr;
  g_armed = true;
  int rc = omega_create(&cfg, 0, &c);
  g_armed = false;
  bad |= check("omega_create (allocation fails)", rc, OMEGA_ENOMEM);
  bad |= c != nullptr;
  // 2) a context (on a box without a GPU omega_create reports OMEGA_EHIP but still hands out the context
  //    to read the message from), then a host-side table build that fails in a std::vector
  rc = omega_create(&cfg, 0, &c);
  std::printf("omega_create: %d (%s)\n", rc, c ? omega_last_error(c) : "-");
  if (!c) return 2;
  double curve[8];
  unsigned char bass[8];
  float comp[8], vsup[8];
  int ranges[4] = {1, 1, 2, 3};
  int bs[2] = {0, 4}, be[2] = {4, 8};
  double sf[2] = {0.6, 0.85};
  for (int i = 0; i < 8; ++i) curve[i] = comp[i] = vsup[i] = 1.0f, bass[i] = 0;
  g_armed = true;
  rc = omega_post_configure(c, 8, curve, bass, comp, comp, vsup, ranges, 6, 7, 0.5f, bs, be, sf, 2);
  g_armed = false;
  bad |= check("omega_post_configure (allocation fails)", rc, OMEGA_ENOMEM);
  bad |= std::strstr(omega_last_error(c), "out of host memory") == nullptr;
  std::printf("message: %s\n", omega_last_error(c));
  omega_destroy(c);
  std::printf(bad ? "FAIL\n" : "ok\n");
  return bad;
}
