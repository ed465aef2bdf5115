// ref_price_driver.cpp — TEST INFRASTRUCTURE. Drives the REFERENCE's own normalize_to_q4, compiled
// from the header where it lies (/root/reference/include/domain/price.hpp:15-29; that header needs
// only <cstdint>/<limits>/<stdexcept>, no generated code or stand-ins). Reads "price scale" pairs on
// stdin and prints "price scale q4" or "price scale EXC <type> <what>" — used by
// tests/golden/make_golden.py to pin the oracle and the product restatement.
#include <cstdio>
#include <stdexcept>

#include "domain/price.hpp"

int main() {
  long long price;
  int scale;
  while (std::scanf("%lld %d", &price, &scale) == 2) {
    try {
      long long q = normalize_to_q4(price, scale);
      std::printf("%lld %d %lld\n", price, scale, q);
    } catch (const std::invalid_argument& e) {
      std::printf("%lld %d EXC invalid_argument %s\n", price, scale, e.what());
    } catch (const std::overflow_error& e) {
      std::printf("%lld %d EXC overflow_error %s\n", price, scale, e.what());
    }
  }
  return 0;
}
