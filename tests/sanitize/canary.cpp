// Sanitizer canaries (test infrastructure, never linked into the product): one deliberate
// heap overflow and one deliberate data race, built with the same flags and loaded the same
// way (ctypes + LD_PRELOAD of the clang runtime) as the sanitized libgpuagg, so
// tests/test_sanitize.py can show that a clean sanitized run means the tool was live.
#include <cstdlib>
#include <thread>

extern "C" int canary_overflow(int i) {
  int *p = (int *)std::malloc(4 * sizeof(int));
  p[0] = 1;
  volatile int v = p[4 + i];  // one past the end (i = 0)
  std::free(p);
  return v;
}

static int shared_counter = 0;

extern "C" int canary_race(int n) {
  auto body = [n] {
    for (int k = 0; k < n; ++k) shared_counter = shared_counter + 1;  // unsynchronised
  };
  std::thread a(body), b(body);
  a.join();
  b.join();
  return shared_counter;
}
