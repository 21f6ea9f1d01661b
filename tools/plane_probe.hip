// Timing probe (not product code): k_round's access pattern at N=65,536 with
// the sender gathers served from a 4-bit LAG plane written beside the 16-bit
// table. The plane is tiled PW members wide (PW = 64/128/256), so one sender
// row segment is PW/2 bytes: at PW = 256 a single 128-B line carries 256
// members where the 16-bit table needs four. The own table stays TW = 64;
// a workgroup covers PW/64 own tiles x RB rows. Trivial merge (nibble min
// + add); writes own 16-bit out and the plane out. Prints ms per launch.
//   hipcc -O3 --offload-arch=gfx950 tools/plane_probe.hip -o build/plane_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned char u8x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pkmax(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, a),
                                                                __builtin_bit_cast(s16x2, b)));
}
__device__ __forceinline__ v4u vmax(v4u a, v4u b) {
  return v4u{pkmax(a.x, b.x), pkmax(a.y, b.y), pkmax(a.z, b.z), pkmax(a.w, b.w)};
}
__device__ __forceinline__ v4u inc(v4u a) { return a + v4u{0x00010001u, 0x00010001u, 0x00010001u, 0x00010001u}; }
// per-nibble unsigned min of two packed 8-nibble words
__device__ __forceinline__ uint32_t nmin(uint32_t a, uint32_t b) {
  const uint32_t lo = 0x0F0F0F0Fu;
  const uint32_t al = a & lo, bl = b & lo, ah = (a >> 4) & lo, bh = (b >> 4) & lo;
  const uint32_t ml = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(
                                                        __builtin_bit_cast(u8x4, al), __builtin_bit_cast(u8x4, bl)));
  const uint32_t mh = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(
                                                        __builtin_bit_cast(u8x4, ah), __builtin_bit_cast(u8x4, bh)));
  return ml | (mh << 4);
}

__global__ void k_init(uint16_t* t, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    t[i] = (uint16_t)(h & 0x3FFF);
  }
}

// MODE 0: senders from the 4-bit plane; MODE 1: senders from the 16-bit
// table (k_round's gathers, for the same WG shape); MODE 2: no senders.
template <int PW, int RB, int MODE, int OTW = 64>
__global__ __launch_bounds__(256) void k_plane(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                               const uint32_t* __restrict__ pin, uint32_t* __restrict__ pout,
                                               const int4* __restrict__ inbox, int n) {
  constexpr int L = PW / 8, RPI = 64 / L;  // lanes per row, rows per wave instruction
  const int nrb = n / RB;
  const int bid = blockIdx.x;
  const int x = bid & 7, j = bid >> 3;
  const int ptile = x + 8 * (j / nrb);
  const int rb = j % nrb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / L, l = lane % L;
  constexpr int TW = OTW;  // own table tile width (64, or PW: one own tile per plane tile)
  const int otile = ptile * (PW / TW) + l / (TW / 8);
  const int64_t oslice = (int64_t)otile * n * TW + (l % (TW / 8)) * 8;
  const int64_t pslice = (int64_t)ptile * n * (PW / 8) + l;  // in dwords
  for (int r = wave * RPI + sub; r < RB; r += 4 * RPI) {
    const int i = rb * RB + r;
    const int64_t o = oslice + (int64_t)i * TW;
    v4u v = *reinterpret_cast<const v4u*>(in + o);
    uint32_t m = 0;
    if constexpr (MODE == 0) {
      const int4 s = inbox[i];
      const uint32_t a = pin[pslice + (int64_t)s.x * (PW / 8)];
      const uint32_t b = pin[pslice + (int64_t)s.y * (PW / 8)];
      const uint32_t c = pin[pslice + (int64_t)s.z * (PW / 8)];
      const uint32_t e = pin[pslice + (int64_t)s.w * (PW / 8)];
      m = nmin(nmin(a, b), nmin(c, e));
      v.x += m & 0x000F000Fu;
      v.y += (m >> 4) & 0x000F000Fu;
      v.z += (m >> 8) & 0x000F000Fu;
      v.w += (m >> 12) & 0x000F000Fu;
    } else if constexpr (MODE == 1) {
      const int4 s = inbox[i];
      const int64_t so = oslice;
      const v4u a = *reinterpret_cast<const v4u*>(in + so + (int64_t)s.x * TW);
      const v4u b = *reinterpret_cast<const v4u*>(in + so + (int64_t)s.y * TW);
      const v4u c = *reinterpret_cast<const v4u*>(in + so + (int64_t)s.z * TW);
      const v4u e = *reinterpret_cast<const v4u*>(in + so + (int64_t)s.w * TW);
      v = vmax(vmax(v, a), vmax(vmax(b, c), e));
    }
    v = inc(v);
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(out + o));
    if constexpr (MODE != 1) {
      const uint32_t w = (v.x & 0xF) | ((v.y & 0xF) << 4) | ((v.z & 0xF) << 8) | ((v.w & 0xF) << 12) |
                         ((v.x >> 16 & 0xF) << 16) | ((v.y >> 16 & 0xF) << 20) | (m & 0xFF000000u);
      __builtin_nontemporal_store(w, pout + pslice + (int64_t)i * (PW / 8));
    }
  }
}

// own table at 8 bits per cell (TW = 256: 256 B per row segment, a lane
// owns 8 cells = 8 B), senders from the 4-bit plane: the byte budget of an
// 8-bit steady-state tier
template <int RB>
__global__ __launch_bounds__(256) void k_own8(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                              const uint32_t* __restrict__ pin, uint32_t* __restrict__ pout,
                                              const int4* __restrict__ inbox, int n) {
  constexpr int PW = 256, L = PW / 8, RPI = 64 / L;
  const int nrb = n / RB;
  const int bid = blockIdx.x;
  const int x = bid & 7, j = bid >> 3;
  const int ptile = x + 8 * (j / nrb);
  const int rb = j % nrb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / L, l = lane % L;
  const int64_t oslice = (int64_t)ptile * n * PW + l * 8;
  const int64_t pslice = (int64_t)ptile * n * (PW / 8) + l;
  for (int r = wave * RPI + sub; r < RB; r += 4 * RPI) {
    const int i = rb * RB + r;
    uint2 v = *reinterpret_cast<const uint2*>(in + oslice + (int64_t)i * PW);
    const int4 s = inbox[i];
    const uint32_t a = pin[pslice + (int64_t)s.x * (PW / 8)];
    const uint32_t b = pin[pslice + (int64_t)s.y * (PW / 8)];
    const uint32_t c = pin[pslice + (int64_t)s.z * (PW / 8)];
    const uint32_t e = pin[pslice + (int64_t)s.w * (PW / 8)];
    const uint32_t m = nmin(nmin(a, b), nmin(c, e));
    v.x += m & 0x0F0F0F0Fu;
    v.y += (m >> 4) & 0x0F0F0F0Fu;
    *reinterpret_cast<uint2*>(out + oslice + (int64_t)i * PW) = v;
    __builtin_nontemporal_store(v.x ^ v.y, pout + pslice + (int64_t)i * (PW / 8));
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 65536;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t cells = (int64_t)n * n;
  uint16_t *t0, *t1;
  uint32_t *p0, *p1;
  int4* inbox;
  CK(hipMalloc(&t0, cells * 2));
  CK(hipMalloc(&t1, cells * 2));
  CK(hipMalloc(&p0, cells / 2));
  CK(hipMalloc(&p1, cells / 2));
  CK(hipMemset(p0, 0x35, cells / 2));
  CK(hipMemset(p1, 0x35, cells / 2));
  CK(hipMalloc(&inbox, (size_t)n * sizeof(int4)));
  std::vector<int4> hin(n);
  uint64_t st = 0x5EED0003ull;
  auto rnd = [&]() {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    return (int)((st >> 33) % (uint64_t)n);
  };
  for (int i = 0; i < n; ++i) hin[i] = int4{rnd(), rnd(), rnd(), rnd()};
  CK(hipMemcpy(inbox, hin.data(), (size_t)n * sizeof(int4), hipMemcpyHostToDevice));
  k_init<<<4096, 256>>>(t0, cells);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto kern, int pw, int rb) {
    const int grid = (n / pw) * (n / rb);
    kern<<<grid, 256>>>(t0, t1, p0, p1, inbox, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) {
      if (r & 1)
        kern<<<grid, 256>>>(t1, t0, p1, p0, inbox, n);
      else
        kern<<<grid, 256>>>(t0, t1, p0, p1, inbox, n);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / reps;
    printf("%-34s %.3f ms/launch   compulsory %.0f GB/s\n", name, per, 4.0 * cells / 1e9 / (per / 1e3));
    fflush(stdout);
  };
  run("16-bit gathers PW=64 RB=256", k_plane<64, 256, 1>, 64, 256);
  run("no senders PW=64 RB=256", k_plane<64, 256, 2>, 64, 256);
  run("no senders PW=256 RB=64", k_plane<256, 64, 2>, 256, 64);
  run("4-bit plane PW=64 RB=256", k_plane<64, 256, 0>, 64, 256);
  run("4-bit plane PW=128 RB=128", k_plane<128, 128, 0>, 128, 128);
  run("4-bit plane PW=128 RB=256", k_plane<128, 256, 0>, 128, 256);
  run("4-bit plane PW=256 RB=64", k_plane<256, 64, 0>, 256, 64);
  run("4-bit plane PW=256 RB=128", k_plane<256, 128, 0>, 256, 128);
  run("4-bit plane PW=256 RB=256", k_plane<256, 256, 0>, 256, 256);
  run("16-bit gathers PW=256 RB=64", k_plane<256, 64, 1>, 256, 64);
  run("own TW=256: no senders RB=64", k_plane<256, 64, 2, 256>, 256, 64);
  run("own TW=256: no senders RB=128", k_plane<256, 128, 2, 256>, 256, 128);
  run("own TW=256: 4-bit PW=256 RB=64", k_plane<256, 64, 0, 256>, 256, 64);
  run("own TW=256: 4-bit PW=256 RB=128", k_plane<256, 128, 0, 256>, 256, 128);
  run("own TW=256: 4-bit PW=256 RB=256", k_plane<256, 256, 0, 256>, 256, 256);
  run("own TW=128: 4-bit PW=128 RB=128", k_plane<128, 128, 0, 128>, 128, 128);
  run("own TW=128: 4-bit PW=256 RB=64", k_plane<256, 64, 0, 128>, 256, 64);
  run("own TW=128: no senders PW=256 RB=64", k_plane<256, 64, 2, 128>, 256, 64);
  run("4-bit plane PW=256 RB=32", k_plane<256, 32, 0>, 256, 32);
  run("4-bit plane PW=256 RB=64 (again)", k_plane<256, 64, 0>, 256, 64);
  run("16-bit gathers PW=64 RB=256", k_plane<64, 256, 1>, 64, 256);
  auto run8 = [&](const char* name, auto kern, int rb) {
    const int grid = (n / 256) * (n / rb);
    uint8_t* a = reinterpret_cast<uint8_t*>(t0);
    uint8_t* b = reinterpret_cast<uint8_t*>(t1);
    kern<<<grid, 256>>>(a, b, p0, p1, inbox, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) {
      if (r & 1)
        kern<<<grid, 256>>>(b, a, p1, p0, inbox, n);
      else
        kern<<<grid, 256>>>(a, b, p0, p1, inbox, n);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-34s %.3f ms/launch\n", name, ms / reps);
    fflush(stdout);
  };
  run8("own 8-bit + 4-bit plane RB=256", k_own8<256>, 256);
  run8("own 8-bit + 4-bit plane RB=128", k_own8<128>, 128);
  run("own TW=256: 4-bit PW=256 RB=256", k_plane<256, 256, 0, 256>, 256, 256);
  return 0;
}
