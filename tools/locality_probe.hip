// Timing probe (not product code): how much of k_round's time is sender-
// segment misses, and does an XCD-resident, sender-phased schedule remove it?
//
// The probe moves exactly k_round's pull-mode bytes with a trivial merge
// (out = max(own, k senders) + 1, packed 16-bit) over a tiled narrow table
// [tile][row][TW] of N rows:
//   A<TW>      k_round's schedule: workgroup = 256 rows x one tile, XCD-aware
//              tile map, own and sender segments loaded per row step.
//   B<TW, P>   persistent: 32 workgroups of 1024 threads per XCD, all of a
//              tile's N rows held in registers by the XCD at once; the k
//              senders merged in P phases by sender row range, so the slice
//              bytes a phase gathers are N/P rows (8 MiB / P at TW = 64).
// Prints ms per launch and a checksum (A and B at one TW must agree).
//   hipcc -O3 --offload-arch=gfx950 tools/locality_probe.hip -o build/locality_probe
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
constexpr int K = 4;

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
__global__ __launch_bounds__(256) void k_a(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                           const int4* __restrict__ inbox, int n, int ntiles) {
  constexpr int SEG = TW / 8, RPW = 64 / SEG, RB = 256;
  const int nrb = n / RB;
  const int bid = blockIdx.x;
  const int x = bid & 7, j = bid >> 3;
  const int tile = x + 8 * (j / nrb);
  const int rb = j % nrb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / SEG, lc = lane % SEG;
  const int64_t slice = (int64_t)tile * n * TW;
  for (int r = wave * RPW + sub; r < RB; r += 4 * RPW) {
    const int i = rb * RB + r;
    const int4 s = inbox[i];
    const int64_t o = slice + (int64_t)i * TW + lc * 8;
    v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(in + o));
    const v4u a = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.x * TW + lc * 8);
    const v4u b = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.y * TW + lc * 8);
    const v4u c = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.z * TW + lc * 8);
    const v4u e = *reinterpret_cast<const v4u*>(in + slice + (int64_t)s.w * TW + lc * 8);
    v = inc(vmax(vmax(v, a), vmax(vmax(b, c), e)));
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(out + o));
  }
}

// 256 workgroups x 1024 threads: XCD x = bid % 8 owns tiles x, x+8, ...;
// workgroup w = bid / 8 holds rows [w*R, (w+1)*R), R = n / 32.
template <int TW, int P>
__global__ __launch_bounds__(1024) void k_b(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                            const int4* __restrict__ inbox, int n, int ntiles) {
  constexpr int SEG = TW / 8;
  constexpr int RPP = 1024 / SEG;        // rows per pass
  const int R = n / 32;
  const int npass = R / RPP;             // 16 (TW 64) or 8 (TW 32) at n = 65,536
  constexpr int MAXP = 16;
  const int x = blockIdx.x & 7, w = blockIdx.x >> 3;
  const int lc = threadIdx.x % SEG, rr = threadIdx.x / SEG;
  int shift = 0;
  while ((n >> shift) > 1) ++shift;      // log2 n
  const int pshift = shift - __builtin_ctz(P);
  // passes 0..7 in registers, 8..15 (TW = 64 only) in LDS
  extern __shared__ v4u s_acc[];
  for (int tile = x; tile < ntiles; tile += 8) {
    const int64_t slice = (int64_t)tile * n * TW;
    v4u acc[8];
#pragma unroll
    for (int q = 0; q < MAXP; ++q)
      if (q < npass) {
        const int i = w * R + q * RPP + rr;
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(in + slice + (int64_t)i * TW + lc * 8));
        if (q < 8)
          acc[q] = v;
        else
          s_acc[(q - 8) * 1024 + threadIdx.x] = v;
      }
#pragma unroll
    for (int ph = 0; ph < P; ++ph) {
#pragma unroll
      for (int q = 0; q < MAXP; ++q)
        if (q < npass) {
          const int i = w * R + q * RPP + rr;
          const int4 s = inbox[i];
          const int sv[4] = {s.x, s.y, s.z, s.w};
          v4u a = q < 8 ? acc[q & 7] : s_acc[(q - 8) * 1024 + threadIdx.x];
#pragma unroll
          for (int t = 0; t < K; ++t)
            if (P == 1 || (sv[t] >> pshift) == ph)
              a = vmax(a, *reinterpret_cast<const v4u*>(in + slice + (int64_t)sv[t] * TW + lc * 8));
          if (q < 8)
            acc[q & 7] = a;
          else
            s_acc[(q - 8) * 1024 + threadIdx.x] = a;
        }
    }
#pragma unroll
    for (int q = 0; q < MAXP; ++q)
      if (q < npass) {
        const int i = w * R + q * RPP + rr;
        const v4u v = q < 8 ? acc[q & 7] : s_acc[(q - 8) * 1024 + threadIdx.x];
        __builtin_nontemporal_store(inc(v), reinterpret_cast<v4u*>(out + slice + (int64_t)i * TW + lc * 8));
      }
  }
}

__global__ void k_sum(const uint16_t* t, int64_t n, unsigned long long* out) {
  unsigned long long s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += (unsigned long long)t[i] * (uint64_t)((i & 1023) + 1);
  atomicAdd(out, s);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 65536;
  const int reps = argc > 2 ? atoi(argv[2]) : 8;
  const int64_t cells = (int64_t)n * n;
  uint16_t *t0, *t1;
  int4* inbox;
  unsigned long long* sum;
  CK(hipMalloc(&t0, cells * 2));
  CK(hipMalloc(&t1, cells * 2));
  CK(hipMalloc(&inbox, (size_t)n * sizeof(int4)));
  CK(hipMalloc(&sum, 8));
  std::vector<int4> hin(n);
  uint64_t st = 0x5EED0003ull;
  auto rnd = [&]() {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    return (int)((st >> 33) % (uint64_t)n);
  };
  for (int i = 0; i < n; ++i) hin[i] = int4{rnd(), rnd(), rnd(), rnd()};
  CK(hipMemcpy(inbox, hin.data(), (size_t)n * sizeof(int4), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  auto run = [&](const char* name, int tw, auto launch) {
    k_init<<<4096, 256>>>(t0, cells);
    CK(hipGetLastError());
    launch(t0, t1);  // warm
    CK(hipDeviceSynchronize());
    CK(hipMemset(sum, 0, 8));
    k_sum<<<4096, 256>>>(t1, cells, sum);
    unsigned long long hs = 0;
    CK(hipMemcpy(&hs, sum, 8, hipMemcpyDeviceToHost));
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) {
      if (r & 1)
        launch(t1, t0);
      else
        launch(t0, t1);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / reps;
    const double alg = 2.0 * cells * (K + 2) / 1e9;
    printf("%-10s tw=%d %.3f ms/launch  alg %.1f GB -> %.0f GB/s  checksum %llx\n", name, tw, per, alg,
           alg / (per / 1e3), hs);
    fflush(stdout);
  };
  const int nt64 = n / 64, nt32 = n / 32;
  CK(hipFuncSetAttribute((const void*)k_b<64, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_b<64, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_b<64, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_b<64, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  run("A", 64, [&](uint16_t* a, uint16_t* b) { k_a<64><<<nt64 * (n / 256), 256>>>(a, b, inbox, n, nt64); });
  run("B_P1", 64, [&](uint16_t* a, uint16_t* b) { k_b<64, 1><<<256, 1024, 131072>>>(a, b, inbox, n, nt64); });
  run("B_P2", 64, [&](uint16_t* a, uint16_t* b) { k_b<64, 2><<<256, 1024, 131072>>>(a, b, inbox, n, nt64); });
  run("B_P4", 64, [&](uint16_t* a, uint16_t* b) { k_b<64, 4><<<256, 1024, 131072>>>(a, b, inbox, n, nt64); });
  run("B_P8", 64, [&](uint16_t* a, uint16_t* b) { k_b<64, 8><<<256, 1024, 131072>>>(a, b, inbox, n, nt64); });
  run("A", 32, [&](uint16_t* a, uint16_t* b) { k_a<32><<<nt32 * (n / 256), 256>>>(a, b, inbox, n, nt32); });
  run("B_P1", 32, [&](uint16_t* a, uint16_t* b) { k_b<32, 1><<<256, 1024>>>(a, b, inbox, n, nt32); });
  run("B_P2", 32, [&](uint16_t* a, uint16_t* b) { k_b<32, 2><<<256, 1024>>>(a, b, inbox, n, nt32); });
  run("B_P4", 32, [&](uint16_t* a, uint16_t* b) { k_b<32, 4><<<256, 1024>>>(a, b, inbox, n, nt32); });
  return 0;
}
