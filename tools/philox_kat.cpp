// Prints philox4x32-10 outputs for (ctr0..3, key0..1) read from argv, using the SAME header
// the HIP kernel includes (gibbs_student_t_amd/csrc/philox.hpp).
#include <cstdio>
#include <cstdlib>

#include "philox.hpp"

int main(int argc, char** argv) {
  if (argc != 7) return 2;
  gst::u32x4 c;
  for (int i = 0; i < 4; ++i) c.v[i] = (uint32_t)strtoul(argv[1 + i], nullptr, 16);
  const uint32_t k0 = (uint32_t)strtoul(argv[5], nullptr, 16);
  const uint32_t k1 = (uint32_t)strtoul(argv[6], nullptr, 16);
  const gst::u32x4 o = gst::philox4x32_10(c, k0, k1);
  std::printf("%08x %08x %08x %08x\n", o.v[0], o.v[1], o.v[2], o.v[3]);
  return 0;
}
