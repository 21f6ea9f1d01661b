// Generates tests/golden/philox_rocrand.json: Philox4x32-10 blocks computed by
// rocRAND's own engine (/opt/rocm/include/rocrand/rocrand_philox4x32_10.h),
// used to pin oracle/philox.{h,py} and the HIP path's Philox. Build+run:
//   hipcc -O1 -o /tmp/gen_philox gen_philox_rocrand.cpp && /tmp/gen_philox > philox_rocrand.json
#include <hip/hip_runtime.h>
#include <rocrand/rocrand_philox4x32_10.h>
#include <cstdio>
#include <cstdint>

int main() {
  // (seed, counter.x, counter.y, counter.z, counter.w)
  const unsigned long long cases[][5] = {
      {0ull, 0, 0, 0, 0},
      {0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF},
      {0x299f31d0a4093822ull, 0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344},
      {0x5EED0001ull, 7, 30, 0x50454552, 0},
      {0x5EED0003ull, 65535, 17, 0x50454552, 0},
      {0x5EED0001ull, 9, 3, 0x504C4143, 0},
      {0xdeadbeefdeadbeefull, 123456, 789, 0, 1},
  };
  printf("[\n");
  const int n = sizeof(cases) / sizeof(cases[0]);
  for (int i = 0; i < n; ++i) {
    unsigned long long seed = cases[i][0];
    unsigned x = (unsigned)cases[i][1], y = (unsigned)cases[i][2];
    unsigned z = (unsigned)cases[i][3], w = (unsigned)cases[i][4];
    // counter = (offset/4 low, offset/4 high, subsequence low, subsequence high)
    unsigned long long subseq = ((unsigned long long)w << 32) | z;
    // advance the 64-bit block counter to T = (y:x) in steps that fit discard()'s
    // 64-bit number-offset (4 numbers per block)
    unsigned long long T = ((unsigned long long)y << 32) | x;
    rocrand_device::philox4x32_10_engine e(seed, subseq, 0);
    for (int q = 0; q < 4; ++q) e.discard((T / 4) * 4ull);
    e.discard((T % 4) * 4ull);
    unsigned o0 = e(), o1 = e(), o2 = e(), o3 = e();
    printf("  {\"key\": [%u, %u], \"ctr\": [%u, %u, %u, %u], \"out\": [%u, %u, %u, %u]}%s\n",
           (unsigned)seed, (unsigned)(seed >> 32), x, y, z, w, o0, o1, o2, o3, i + 1 < n ? "," : "");
  }
  printf("]\n");
  return 0;
}
