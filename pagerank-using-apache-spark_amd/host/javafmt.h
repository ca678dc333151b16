// Java Double.toString for the output writers (Sparky.java:237 saveAsTextFile of Tuple2<String,
// Double>; the north_star "<url> has rank: <r>." line).  Shortest uniquely-distinguishing digits
// (JDK 19+ algorithm, via std::to_chars), at least two significant digits, decimal layout for
// 1e-3 <= |x| < 1e7 and "d.dddE<n>" otherwise.
#pragma once

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace pr_host {

// Writes into buf (>= 40 bytes); returns the length.
inline size_t java_double_to_string(double x, char *buf) {
  if (std::isnan(x)) { std::memcpy(buf, "NaN", 3); return 3; }
  if (std::isinf(x)) {
    if (x > 0) { std::memcpy(buf, "Infinity", 8); return 8; }
    std::memcpy(buf, "-Infinity", 9);
    return 9;
  }
  if (x == 0.0) {
    if (std::signbit(x)) { std::memcpy(buf, "-0.0", 4); return 4; }
    std::memcpy(buf, "0.0", 3);
    return 3;
  }
  size_t o = 0;
  if (x < 0) { buf[o++] = '-'; x = -x; }
  // shortest round-trip digits in scientific form: d[.ddd]e±XX
  char tmp[64];
  auto res = std::to_chars(tmp, tmp + sizeof(tmp), x, std::chars_format::scientific);
  *res.ptr = '\0';
  char digits[32];
  int nd = 0;
  const char *p = tmp;
  for (; *p && *p != 'e'; ++p)
    if (*p != '.') digits[nd++] = *p;
  int e10 = std::atoi(p + 1);
  while (nd > 1 && digits[nd - 1] == '0') --nd;
  if (nd == 1) {
    // JDK 19+: two significant digits, the 2-digit decimal closest to x
    char t2[32];
    std::snprintf(t2, sizeof(t2), "%.1e", x);
    digits[0] = t2[0];
    digits[1] = t2[2];
    e10 = std::atoi(t2 + 4);
    nd = (digits[1] == '0') ? 1 : 2;
  }
  const int point = e10 + 1;  // value = 0.d1d2... * 10^point
  if (x >= 1e-3 && x < 1e7) {
    if (point <= 0) {
      buf[o++] = '0';
      buf[o++] = '.';
      for (int k = 0; k < -point; ++k) buf[o++] = '0';
      for (int k = 0; k < nd; ++k) buf[o++] = digits[k];
    } else if (point >= nd) {
      for (int k = 0; k < nd; ++k) buf[o++] = digits[k];
      for (int k = nd; k < point; ++k) buf[o++] = '0';
      buf[o++] = '.';
      buf[o++] = '0';
    } else {
      for (int k = 0; k < point; ++k) buf[o++] = digits[k];
      buf[o++] = '.';
      for (int k = point; k < nd; ++k) buf[o++] = digits[k];
    }
    return o;
  }
  buf[o++] = digits[0];
  buf[o++] = '.';
  if (nd == 1) buf[o++] = '0';
  for (int k = 1; k < nd; ++k) buf[o++] = digits[k];
  buf[o++] = 'E';
  o += (size_t)std::snprintf(buf + o, 16, "%d", e10);
  return o;
}

}  // namespace pr_host
