// Test helper: reads one IEEE-754 bit pattern (hex) per line, prints Java Double.toString.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "javafmt.h"

int main() {
  char line[64], out[64];
  while (std::fgets(line, sizeof line, stdin)) {
    unsigned long long bits = 0;
    if (std::sscanf(line, "%llx", &bits) != 1) continue;
    double x;
    std::memcpy(&x, &bits, sizeof x);
    const size_t n = pr_host::java_double_to_string(x, out);
    std::fwrite(out, 1, n, stdout);
    std::fputc('\n', stdout);
  }
  return 0;
}
