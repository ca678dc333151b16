// Driver of the IPC protocol's CPU model checker (host/ipc_model.cpp) for the sanitizer builds of
// tests/test_sanitizers_cpu.py: P ranks as threads over the shared-page model, every op sequence
// checked; the sanitizers watch the checker and the protocol template (pr_ipc_protocol.h) itself.
#include <cstdint>
#include <initializer_list>
#include <cstdio>
extern "C" int64_t ipc_model_run(int P, int nc, int n_ops, uint64_t seed, int max_delay_us, char *err, int errlen);
extern "C" int64_t ipc_model_run2(int P, int nc, int n_ops, uint64_t seed, int max_delay_us, int reenable_one_in,
                                  char *err, int errlen);
int main() {
  char err[512];
  int bad = 0;
  for (int P : {2, 3, 8})
    for (int nc : {1, 4, 8})
      for (uint64_t seed : {1ull, 7ull}) {
        const int64_t w = ipc_model_run(P, nc, 60, seed, 50, err, sizeof err);
        if (w < 0) { std::printf("P=%d nc=%d seed=%llu: %s\n", P, nc, (unsigned long long)seed, err); ++bad; }
      }
  // past three event generations per buffer, with re-enables (the generation helper, pr_ipc_gens.h)
  for (int P : {2, 4}) {
    const int64_t w = ipc_model_run2(P, 8, 240, 11, 5, 20, err, sizeof err);
    if (w < 0) { std::printf("generations P=%d: %s\n", P, err); ++bad; }
  }
  std::printf("done, %d failures\n", bad);
  return bad != 0;
}
