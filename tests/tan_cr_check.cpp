// Host build of csrc/sk_tan_cr.hpp for tests/test_tan_cr_cpu.py: reads
// little-endian doubles on stdin, writes tan_cr of each on stdout.
#include <stdio.h>

#include "../skillshot_learning_amd/csrc/sk_tan_cr.hpp"

int main() {
  double x;
  while (fread(&x, sizeof x, 1, stdin) == 1) {
    double t = sktan::tan_cr(x);
    fwrite(&t, sizeof t, 1, stdout);
  }
  return 0;
}
