// Histogram-kernel microbenchmark (standalone): variants of the LDS-privatised
// row-major histogram on packed uint8 group bins, timed with hipEvents.
// Build: hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics scripts/hist_micro.hip -o build/hist_micro
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);           \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int G = 28, NB = 256, SD = 7;  // groups, bins per group, dwords per row
constexpr int TB = G * NB;

// A: baseline - interleaved (g,h), one row per thread-iteration
__global__ __launch_bounds__(512) void hA(const uint32_t* rows, const float2* gh, const int* idx, int n, int nb,
                                         float* slab) {
  __shared__ float lds[2 * TB];
  for (int i = threadIdx.x; i < 2 * TB; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  int chunk = (n + nb - 1) / nb, rb = blockIdx.x * chunk, re = min(n, rb + chunk);
  int tpr = SD, rpi = blockDim.x / tpr, myr = threadIdx.x / tpr, myd = threadIdx.x - myr * tpr;
  if (myr < rpi) {
    for (int p = rb + myr; p < re; p += rpi) {
      int row = idx ? idx[p] : p;
      uint32_t w = rows[(size_t)row * SD + myd];
      float2 v = gh[row];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t b = (w >> (8 * k)) & 255u;
        if (b) {
          int o = (myd * 4 + k) * NB + b;
          atomicAdd(&lds[2 * o], v.x);
          atomicAdd(&lds[2 * o + 1], v.y);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * TB; i += blockDim.x) slab[(size_t)blockIdx.x * 2 * TB + i] = lds[i];
}

// B/C/D: split g and h arrays, R rows per thread-iteration with loads batched
template <int R>
__global__ __launch_bounds__(512) void hB(const uint32_t* rows, const float2* gh, const int* idx, int n, int nb,
                                         float* slab) {
  __shared__ float lg[TB];
  __shared__ float lh[TB];
  for (int i = threadIdx.x; i < TB; i += blockDim.x) lg[i] = lh[i] = 0.f;
  __syncthreads();
  int chunk = (n + nb - 1) / nb, rb = blockIdx.x * chunk, re = min(n, rb + chunk);
  int tpr = SD, rpi = blockDim.x / tpr, myr = threadIdx.x / tpr, myd = threadIdx.x - myr * tpr;
  if (myr < rpi) {
    for (int p0 = rb + myr; p0 < re; p0 += rpi * R) {
      int rr[R];
      uint32_t w[R];
      float2 v[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        int p = p0 + j * rpi;
        rr[j] = p < re ? (idx ? idx[p] : p) : -1;
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        if (rr[j] >= 0) {
          w[j] = rows[(size_t)rr[j] * SD + myd];
          v[j] = gh[rr[j]];
        } else {
          w[j] = 0;
          v[j] = make_float2(0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t b = (w[j] >> (8 * k)) & 255u;
          if (b) {
            int o = (myd * 4 + k) * NB + b;
            atomicAdd(&lg[o], v[j].x);
            atomicAdd(&lh[o], v[j].y);
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TB; i += blockDim.x) {
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i] = lg[i];
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i + 1] = lh[i];
  }
}

// E: like C but 256-thread blocks (more blocks per CU)
template <int R>
__global__ __launch_bounds__(256) void hE(const uint32_t* rows, const float2* gh, const int* idx, int n, int nb,
                                         float* slab) {
  __shared__ float lg[TB];
  __shared__ float lh[TB];
  for (int i = threadIdx.x; i < TB; i += blockDim.x) lg[i] = lh[i] = 0.f;
  __syncthreads();
  int chunk = (n + nb - 1) / nb, rb = blockIdx.x * chunk, re = min(n, rb + chunk);
  int tpr = SD, rpi = blockDim.x / tpr, myr = threadIdx.x / tpr, myd = threadIdx.x - myr * tpr;
  if (myr < rpi) {
    for (int p0 = rb + myr; p0 < re; p0 += rpi * R) {
      int rr[R];
      uint32_t w[R];
      float2 v[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        int p = p0 + j * rpi;
        rr[j] = p < re ? (idx ? idx[p] : p) : -1;
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        w[j] = rr[j] >= 0 ? rows[(size_t)rr[j] * SD + myd] : 0u;
        v[j] = rr[j] >= 0 ? gh[rr[j]] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t b = (w[j] >> (8 * k)) & 255u;
          if (b) {
            int o = (myd * 4 + k) * NB + b;
            atomicAdd(&lg[o], v[j].x);
            atomicAdd(&lh[o], v[j].y);
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TB; i += blockDim.x) {
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i] = lg[i];
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i + 1] = lh[i];
  }
}

// F: no atomics at all (bandwidth ceiling of the loads): sum into registers
template <int R>
__global__ __launch_bounds__(512) void hF(const uint32_t* rows, const float2* gh, const int* idx, int n, int nb,
                                         float* slab) {
  int chunk = (n + nb - 1) / nb, rb = blockIdx.x * chunk, re = min(n, rb + chunk);
  int tpr = SD, rpi = blockDim.x / tpr, myr = threadIdx.x / tpr, myd = threadIdx.x - myr * tpr;
  float acc = 0.f;
  if (myr < rpi) {
    for (int p0 = rb + myr; p0 < re; p0 += rpi * R) {
      int rr[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        int p = p0 + j * rpi;
        rr[j] = p < re ? (idx ? idx[p] : p) : -1;
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        if (rr[j] >= 0) {
          uint32_t w = rows[(size_t)rr[j] * SD + myd];
          float2 v = gh[rr[j]];
          acc += (float)(w & 255u) * v.x + v.y;
        }
      }
    }
  }
  if (acc == 12345.f) slab[threadIdx.x] = acc;
}


// G: int32 fixed point, two ds_add_u32 per group-row
template <int R>
__global__ __launch_bounds__(512) void hG(const uint32_t* rows, const float2* gh, const int* idx, int n, int nb,
                                         float* slab) {
  __shared__ int lg[TB];
  __shared__ int lh[TB];
  for (int i = threadIdx.x; i < TB; i += blockDim.x) lg[i] = lh[i] = 0;
  __syncthreads();
  int chunk = (n + nb - 1) / nb, rb = blockIdx.x * chunk, re = min(n, rb + chunk);
  const float sg = 65536.f, sh = 65536.f;
  int tpr = SD, rpi = blockDim.x / tpr, myr = threadIdx.x / tpr, myd = threadIdx.x - myr * tpr;
  if (myr < rpi) {
    for (int p0 = rb + myr; p0 < re; p0 += rpi * R) {
      int rr[R];
      uint32_t w[R];
      float2 v[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        int p = p0 + j * rpi;
        rr[j] = p < re ? (idx ? idx[p] : p) : -1;
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        w[j] = rr[j] >= 0 ? rows[(size_t)rr[j] * SD + myd] : 0u;
        v[j] = rr[j] >= 0 ? gh[rr[j]] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        int ig = __float2int_rn(v[j].x * sg), ih = __float2int_rn(v[j].y * sh);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t b = (w[j] >> (8 * k)) & 255u;
          if (b) {
            int o = (myd * 4 + k) * NB + b;
            atomicAdd(&lg[o], ig);
            atomicAdd(&lh[o], ih);
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TB; i += blockDim.x) {
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i] = lg[i] / sg;
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i + 1] = lh[i] / sh;
  }
}

// I: packed 64-bit (g int32 high | h uint32 low), ONE ds_add_u64 per group-row
template <int R>
__global__ __launch_bounds__(512) void hI(const uint32_t* rows, const float2* gh, const int* idx, int n, int nb,
                                         float* slab) {
  extern __shared__ unsigned long long l64[];
  for (int i = threadIdx.x; i < TB; i += blockDim.x) l64[i] = 0ull;
  __syncthreads();
  int chunk = (n + nb - 1) / nb, rb = blockIdx.x * chunk, re = min(n, rb + chunk);
  const float sg = 65536.f, sh = 65536.f;
  int tpr = SD, rpi = blockDim.x / tpr, myr = threadIdx.x / tpr, myd = threadIdx.x - myr * tpr;
  if (myr < rpi) {
    for (int p0 = rb + myr; p0 < re; p0 += rpi * R) {
      int rr[R];
      uint32_t w[R];
      float2 v[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        int p = p0 + j * rpi;
        rr[j] = p < re ? (idx ? idx[p] : p) : -1;
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        w[j] = rr[j] >= 0 ? rows[(size_t)rr[j] * SD + myd] : 0u;
        v[j] = rr[j] >= 0 ? gh[rr[j]] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        long long ig = __float2int_rn(v[j].x * sg);
        unsigned long long ih = (unsigned)__float2int_rn(v[j].y * sh);
        unsigned long long pk = (static_cast<unsigned long long>(ig) << 32) + ih;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t b = (w[j] >> (8 * k)) & 255u;
          if (b) {
            int o = (myd * 4 + k) * NB + b;
            atomicAdd(&l64[o], pk);
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TB; i += blockDim.x) {
    unsigned long long x = l64[i];
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i] = (int)(x >> 32) / sg;
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i + 1] = (unsigned)(x & 0xffffffffu) / sh;
  }
}

// J: int64 two ds_add_u64 per group-row (dynamic LDS 16 B/bin)
template <int R>
__global__ __launch_bounds__(512) void hJ(const uint32_t* rows, const float2* gh, const int* idx, int n, int nb,
                                         float* slab) {
  extern __shared__ unsigned long long l64[];
  unsigned long long* lg = l64;
  unsigned long long* lh = l64 + TB;
  for (int i = threadIdx.x; i < 2 * TB; i += blockDim.x) l64[i] = 0ull;
  __syncthreads();
  int chunk = (n + nb - 1) / nb, rb = blockIdx.x * chunk, re = min(n, rb + chunk);
  const double sg = 1099511627776.0, sh = 1099511627776.0;
  int tpr = SD, rpi = blockDim.x / tpr, myr = threadIdx.x / tpr, myd = threadIdx.x - myr * tpr;
  if (myr < rpi) {
    for (int p0 = rb + myr; p0 < re; p0 += rpi * R) {
      int rr[R];
      uint32_t w[R];
      float2 v[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        int p = p0 + j * rpi;
        rr[j] = p < re ? (idx ? idx[p] : p) : -1;
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        w[j] = rr[j] >= 0 ? rows[(size_t)rr[j] * SD + myd] : 0u;
        v[j] = rr[j] >= 0 ? gh[rr[j]] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        unsigned long long ig = (unsigned long long)__double2ll_rn(v[j].x * sg);
        unsigned long long ih = (unsigned long long)__double2ll_rn(v[j].y * sh);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t b = (w[j] >> (8 * k)) & 255u;
          if (b) {
            int o = (myd * 4 + k) * NB + b;
            atomicAdd(&lg[o], ig);
            atomicAdd(&lh[o], ih);
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TB; i += blockDim.x) {
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i] = (long long)lg[i] / sg;
    slab[(size_t)blockIdx.x * 2 * TB + 2 * i + 1] = (long long)lh[i] / sh;
  }
}

__global__ void reduce(const float* slab, int nb, double* out) {
  int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= 2 * TB) return;
  double s = 0;
  for (int p = 0; p < nb; ++p) s += slab[(size_t)p * 2 * TB + v];
  out[v] = s;
}

typedef void (*KFn)(const uint32_t*, const float2*, const int*, int, int, float*);

int g_dyn = 0;
float TimeIt(KFn fn, int threads, const uint32_t* rows, const float2* gh, const int* idx, int n, int nb, float* slab,
             int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  fn<<<nb, threads, g_dyn>>>(rows, gh, idx, n, nb, slab);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) fn<<<nb, threads, g_dyn>>>(rows, gh, idx, n, nb, slab);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return 1000.f * ms / reps;
}

int main() {
  const int N = 10000000;
  std::mt19937 rng(1);
  std::vector<uint32_t> h_rows((size_t)N * SD);
  std::vector<float2> h_gh(N);
  for (size_t i = 0; i < h_rows.size(); ++i) {
    uint32_t w = 0;
    for (int k = 0; k < 4; ++k) {
      uint32_t b = rng() % 256;
      if ((rng() & 3) == 0) b = 0;  // 25% at the implicit most-frequent bin
      w |= b << (8 * k);
    }
    h_rows[i] = w;
  }
  for (int i = 0; i < N; ++i) h_gh[i] = make_float2((rng() % 1000) / 1000.f - 0.5f, (rng() % 1000) / 4000.f);
  std::vector<int> h_idx;
  for (int i = 0; i < N; ++i)
    if (rng() % 2) h_idx.push_back(i);
  uint32_t* rows;
  float2* gh;
  int* idx;
  float* slab;
  CK(hipMalloc(&rows, h_rows.size() * 4));
  CK(hipMalloc(&gh, (size_t)N * 8));
  CK(hipMalloc(&idx, h_idx.size() * 4));
  CK(hipMalloc(&slab, (size_t)4096 * 2 * TB * 4));
  CK(hipMemcpy(rows, h_rows.data(), h_rows.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(gh, h_gh.data(), (size_t)N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(idx, h_idx.data(), h_idx.size() * 4, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)hJ<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * TB * 8));
  struct V {
    const char* name;
    KFn fn;
    int threads;
    int dyn;
  } vs[] = {{"A base f32", hA, 512, 0},        {"C f32 R4", hB<4>, 512, 0},   {"G i32 R4", hG<4>, 512, 0},
            {"I pk64 R4", hI<4>, 512, TB * 8}, {"J i64x2 R4", hJ<4>, 512, 2 * TB * 8},
            {"F noatomic R4", hF<4>, 512, 0}};
  struct Case {
    const char* name;
    bool use_idx;
    int n;
  } cs[] = {{"root 10M", false, N}, {"gather 5M", true, (int)h_idx.size()}, {"gather 200K", true, 200000},
            {"gather 20K", true, 20000}, {"gather 2K", true, 2000}};
  for (auto& c : cs) {
    for (int nbmode = 0; nbmode < 3; ++nbmode) {
      int rows_per_block = nbmode == 0 ? 2048 : (nbmode == 1 ? 8192 : 512);
      int nb = std::max(1, std::min(nbmode == 2 ? 2048 : 512, (c.n + rows_per_block - 1) / rows_per_block));
      for (auto& v : vs) {
        g_dyn = v.dyn;
        float us = TimeIt(v.fn, v.threads, rows, gh, c.use_idx ? idx : nullptr, c.n, nb, slab, 10);
        double gbs = (double)c.n * (SD * 4 + 8 + (c.use_idx ? 4 : 0)) / (us * 1e3);
        printf("%-12s nb=%5d %-14s %9.1f us  %7.1f GB/s\n", c.name, nb, v.name, us, gbs);
      }
    }
  }
  return 0;
}
