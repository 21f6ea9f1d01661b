// Timing probe (not product code): k_round's access pattern at N=65,536,
// TW=64 against (a) the stream floor (own segment in, own segment out, no
// sender gathers: the HBM floor for the round's compulsory bytes) and (b)
// sender gathers from a compact snapshot plane written beside the table
// (4-bit or 8-bit per cell, so a tile's sender slice is 2 or 4 MiB and fits
// an XCD's L2). Trivial merge; prints ms per launch.
//   hipcc -O3 --offload-arch=gfx950 tools/snapshot_probe.hip -o build/snapshot_probe
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
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
constexpr int RB = 256;

__device__ __forceinline__ uint32_t pkmax(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, a),
                                                                __builtin_bit_cast(s16x2, b)));
}
__device__ __forceinline__ v4u vmax(v4u a, v4u b) {
  return v4u{pkmax(a.x, b.x), pkmax(a.y, b.y), pkmax(a.z, b.z), pkmax(a.w, b.w)};
}
__device__ __forceinline__ v4u inc(v4u a) { return a + v4u{0x00010001u, 0x00010001u, 0x00010001u, 0x00010001u}; }

__global__ void k_init(uint16_t* t, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    t[i] = (uint16_t)(h & 0x3FFF);
  }
}

template <int TW>
__device__ __forceinline__ void coords(int n, int& tile, int& rb) {
  const int nrb = n / RB;
  const int bid = blockIdx.x;
  const int x = bid & 7, j = bid >> 3;
  tile = x + 8 * (j / nrb);
  rb = j % nrb;
}

// MODE 0: k_round's gathers from the 16-bit table; 1: floor (no senders);
// 2: 4-bit snapshot plane; 3: 8-bit snapshot plane; 4: senders = the own row
// (cache hits: issue cost); 5: senders = the next 4 rows; 6/7: 1 / 2 random
// senders
template <int MODE, int TW = 64>
__global__ __launch_bounds__(256) void k_probe(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                               const uint8_t* __restrict__ sin, uint8_t* __restrict__ sout,
                                               const int4* __restrict__ inbox, int n) {
  constexpr int SEG = TW / 8, RPW = 64 / SEG;
  int tile, rb;
  coords<TW>(n, tile, rb);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / SEG, lc = lane % SEG;
  const int64_t slice = (int64_t)tile * n * TW;
  for (int r = wave * RPW + sub; r < RB; r += 4 * RPW) {
    const int i = rb * RB + r;
    const int64_t o = slice + (int64_t)i * TW + lc * 8;
    v4u v = *reinterpret_cast<const v4u*>(in + o);
    if constexpr (MODE == 0 || MODE == 4 || MODE == 5) {
      int4 s = inbox[i];
      if (MODE == 4) s = int4{i, i, i, i};
      if (MODE == 5) s = int4{(i + 1) % n, (i + 2) % n, (i + 3) % n, (i + 4) % n};
      const v4u a = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.x * TW + lc * 8);
      const v4u b = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.y * TW + lc * 8);
      const v4u c = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.z * TW + lc * 8);
      const v4u e = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.w * TW + lc * 8);
      v = vmax(vmax(v, a), vmax(vmax(b, c), e));
    } else if constexpr (MODE == 6 || MODE == 7) {
      const int4 s = inbox[i];
      const v4u a = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.x * TW + lc * 8);
      v = vmax(v, a);
      if (MODE == 7) v = vmax(v, *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.y * TW + lc * 8));
    } else if constexpr (MODE == 2 || MODE == 9) {
      // 4 bits per cell: a lane's 8 cells are one dword; a row segment 32 B
      const int4 s = inbox[i];
      const int64_t ss = (int64_t)tile * n * (TW / 2) + lc * 4;
      const uint32_t a = *reinterpret_cast<const uint32_t*>(sin + ss + (int64_t)s.x * (TW / 2));
      const uint32_t b = *reinterpret_cast<const uint32_t*>(sin + ss + (int64_t)s.y * (TW / 2));
      const uint32_t c = *reinterpret_cast<const uint32_t*>(sin + ss + (int64_t)s.z * (TW / 2));
      const uint32_t e = *reinterpret_cast<const uint32_t*>(sin + ss + (int64_t)s.w * (TW / 2));
      const uint32_t m = __builtin_elementwise_max(__builtin_elementwise_max(a, b), __builtin_elementwise_max(c, e));
      v.x += m & 0x000F000Fu;
      v.y += (m >> 4) & 0x000F000Fu;
      v.z += (m >> 8) & 0x000F000Fu;
      v.w += (m >> 12) & 0x000F000Fu;
      if (MODE == 2)
        *reinterpret_cast<uint32_t*>(sout + (int64_t)tile * n * (TW / 2) + (int64_t)i * (TW / 2) + lc * 4) =
            (v.x & 0xF) | ((v.y & 0xF) << 4) | ((v.z & 0xF) << 8) | ((v.w & 0xF) << 12) | (m & 0xFFFF0000u);
    } else if constexpr (MODE == 3) {
      const int4 s = inbox[i];
      const int64_t ss = (int64_t)tile * n * TW + lc * 8;
      const v2u a = *reinterpret_cast<const v2u*>(sin + ss + (int64_t)s.x * TW);
      const v2u b = *reinterpret_cast<const v2u*>(sin + ss + (int64_t)s.y * TW);
      const v2u c = *reinterpret_cast<const v2u*>(sin + ss + (int64_t)s.z * TW);
      const v2u e = *reinterpret_cast<const v2u*>(sin + ss + (int64_t)s.w * TW);
      const v2u m = v2u{a.x ^ b.x ^ c.x ^ e.x, a.y ^ b.y ^ c.y ^ e.y};
      v.x += m.x & 0x00FF00FFu;
      v.y += m.y & 0x00FF00FFu;
      *reinterpret_cast<v2u*>(sout + (int64_t)tile * n * TW + (int64_t)i * TW + lc * 8) = v2u{v.x ^ v.z, v.y ^ v.w};
    }
    __builtin_nontemporal_store(inc(v), reinterpret_cast<v4u*>(out + o));
  }
}

// two row steps in flight per wave (10 loads issued before the first use)
template <int TW = 64>
__global__ __launch_bounds__(256) void k_pipe2(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                               const uint8_t* __restrict__, uint8_t* __restrict__,
                                               const int4* __restrict__ inbox, int n) {
  constexpr int SEG = TW / 8, RPW = 64 / SEG;
  int tile, rb;
  coords<TW>(n, tile, rb);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / SEG, lc = lane % SEG;
  const int64_t slice = (int64_t)tile * n * TW;
  for (int r = wave * RPW + sub; r < RB; r += 8 * RPW) {
    const int i0 = rb * RB + r, i1 = i0 + 4 * RPW;
    const int4 s0 = inbox[i0], s1 = inbox[i1];
    const int64_t o0 = slice + (int64_t)i0 * TW + lc * 8, o1 = slice + (int64_t)i1 * TW + lc * 8;
    v4u v0 = *reinterpret_cast<const v4u*>(in + o0);
    v4u v1 = *reinterpret_cast<const v4u*>(in + o1);
    const v4u a0 = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s0.x * TW + lc * 8);
    const v4u b0 = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s0.y * TW + lc * 8);
    const v4u c0 = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s0.z * TW + lc * 8);
    const v4u e0 = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s0.w * TW + lc * 8);
    const v4u a1 = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s1.x * TW + lc * 8);
    const v4u b1 = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s1.y * TW + lc * 8);
    const v4u c1 = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s1.z * TW + lc * 8);
    const v4u e1 = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s1.w * TW + lc * 8);
    v0 = vmax(vmax(v0, a0), vmax(vmax(b0, c0), e0));
    v1 = vmax(vmax(v1, a1), vmax(vmax(b1, c1), e1));
    __builtin_nontemporal_store(inc(v0), reinterpret_cast<v4u*>(out + o0));
    __builtin_nontemporal_store(inc(v1), reinterpret_cast<v4u*>(out + o1));
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 65536;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t cells = (int64_t)n * n;
  uint16_t *t0, *t1;
  uint8_t *s0, *s1;
  int4* inbox;
  CK(hipMalloc(&t0, cells * 2));
  CK(hipMalloc(&t1, cells * 2));
  CK(hipMalloc(&s0, cells));
  CK(hipMalloc(&s1, cells));
  CK(hipMemset(s0, 0x11, cells));
  CK(hipMemset(s1, 0x11, cells));
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
  auto run = [&](const char* name, auto kern, int TW = 64) {
    const int grid = (n / TW) * (n / RB);
    kern<<<grid, 256>>>(t0, t1, s0, s1, inbox, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) {
      if (r & 1)
        kern<<<grid, 256>>>(t1, t0, s1, s0, inbox, n);
      else
        kern<<<grid, 256>>>(t0, t1, s0, s1, inbox, n);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / reps;
    printf("%-28s %.3f ms/launch   compulsory %.0f GB/s\n", name, per, 4.0 * cells / 1e9 / (per / 1e3));
    fflush(stdout);
  };
  run("gather 16-bit (k_round)", k_probe<0>);
  run("stream floor (no senders)", k_probe<1>);
  run("gather 4-bit snapshot", k_probe<2>);
  run("gather 8-bit snapshot", k_probe<3>);
  run("2 row steps in flight", k_pipe2<64>);
  run("4-bit snapshot, read-only", k_probe<9>);
  run("senders = own row", k_probe<4>);
  run("senders = next 4 rows", k_probe<5>);
  run("1 random sender", k_probe<6>);
  run("2 random senders", k_probe<7>);
  run("gather 16-bit TW=128", k_probe<0, 128>, 128);
  run("stream floor TW=128", k_probe<1, 128>, 128);
  run("gather 16-bit TW=256", k_probe<0, 256>, 256);
  run("gather 16-bit TW=32", k_probe<0, 32>, 32);
  run("gather 16-bit (k_round)", k_probe<0>);
  return 0;
}
