// Microbenchmark: the memory pattern of the C2 Hogwild epoch without its arithmetic, to bound what
// bmf_sgd_hogwild_kernel can reach.  100 M ratings (users uniform over 1 M, items Zipf(0.8) over
// 100 k), k = 64 fp32 rows (256 B), 16 lanes per rating, 8,192 waves each walking a contiguous
// chunk of the stream, like the kernel.  Modes:
//   0  read U_u and V_i rows (gather only)
//   1  read both rows, write both back (the epoch's row traffic: 1,024 B per rating)
//   2  mode 1 + the 4-B bias reads and writes and the 12-B stream read (1,052 B, the kernel's
//      algorithmic bytes)
//   3  mode 1 + bias reads only;  4  mode 1 + bias writes only;  5  mode 2 with nontemporal bias
//      stores
// hipcc --offload-arch=gfx950 -O3 -o rowrmw rowrmw.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void rmw(const int* __restrict__ su, const int* __restrict__ si,
                                           const float* __restrict__ sr, long long n,
                                           long long chunk, float4* U, float4* V, float* bu,
                                           float* bi) {
    const int lane = threadIdx.x & 63, sub = lane / 16, q = lane % 16;
    const long long wave = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long begin = wave * chunk, end = min(begin + chunk, n);
    for (long long base = begin; base < end; base += 64) {
        const long long x = base + lane;
        const int my_u = x < end ? su[x] : 0, my_i = x < end ? si[x] : 0;
        const float my_r = x < end ? sr[x] : 0.f;
        asm volatile("" ::"v"(my_u), "v"(my_i), "v"(my_r));
        const int cnt = (int)min(64LL, end - base);
        for (int step = 0; step < cnt; step += 4) {
            const int u = __shfl(my_u, step + sub), i = __shfl(my_i, step + sub);
            const float r = __shfl(my_r, step + sub);
            if (step + sub >= cnt) continue;
            float4 a = U[(long long)u * 16 + q], b = V[(long long)i * 16 + q];
            float s = a.x + b.y + r;
            if (MODE == 2 || MODE == 3 || MODE == 5) s += bu[u] + bi[i];
            if (MODE == 0) {
                if (s == 12345.f) U[0] = a;  // keep the loads
                continue;
            }
            a.x += 1e-30f * s;
            b.x += 1e-30f * s;
            U[(long long)u * 16 + q] = a;
            V[(long long)i * 16 + q] = b;
            if ((MODE == 2 || MODE == 4) && q == 0) {
                bu[u] = s;
                bi[i] = s;
            }
            if (MODE == 5 && q == 0) {
                __builtin_nontemporal_store(s, bu + u);
                __builtin_nontemporal_store(s, bi + i);
            }
        }
    }
}

int main() {
    const long long n = 100000000, nu = 1000000, ni = 100000;
    std::vector<int> hu(n), hi(n);
    std::vector<float> hr(n, 3.0f);
    std::vector<double> cdf(ni);
    double acc = 0;
    for (long long i = 0; i < ni; ++i) cdf[i] = (acc += std::pow((double)(i + 1), -0.8));
    for (auto& c : cdf) c /= acc;
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> U01(0, 1);
    for (long long x = 0; x < n; ++x) {
        hu[x] = (int)(g() % nu);
        hi[x] = (int)std::min<long long>(ni - 1, std::lower_bound(cdf.begin(), cdf.end(), U01(g)) - cdf.begin());
    }
    int *du, *di;
    float *dr, *bu, *bi;
    float4 *U, *V;
    CK(hipMalloc(&du, n * 4));
    CK(hipMalloc(&di, n * 4));
    CK(hipMalloc(&dr, n * 4));
    CK(hipMalloc(&U, nu * 256));
    CK(hipMalloc(&V, ni * 256));
    CK(hipMalloc(&bu, nu * 4));
    CK(hipMalloc(&bi, ni * 4));
    CK(hipMemcpy(du, hu.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(di, hi.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, hr.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(U, 0, nu * 256));
    CK(hipMemset(V, 0, ni * 256));
    CK(hipMemset(bu, 0, nu * 4));
    CK(hipMemset(bi, 0, ni * 4));
    const long long waves = 8192, chunk = (n + waves - 1) / waves;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes[6] = {512.0, 1024.0, 1052.0, 1032.0, 1032.0, 1052.0};
    for (int mode = 0; mode < 6; ++mode) {
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipEventRecord(e0));
            if (mode == 0) rmw<0><<<waves / 4, 256>>>(du, di, dr, n, chunk, U, V, bu, bi);
            if (mode == 1) rmw<1><<<waves / 4, 256>>>(du, di, dr, n, chunk, U, V, bu, bi);
            if (mode == 2) rmw<2><<<waves / 4, 256>>>(du, di, dr, n, chunk, U, V, bu, bi);
            if (mode == 3) rmw<3><<<waves / 4, 256>>>(du, di, dr, n, chunk, U, V, bu, bi);
            if (mode == 4) rmw<4><<<waves / 4, 256>>>(du, di, dr, n, chunk, U, V, bu, bi);
            if (mode == 5) rmw<5><<<waves / 4, 256>>>(du, di, dr, n, chunk, U, V, bu, bi);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0)
                std::printf("mode %d: %.2f ms, %.2f G ratings/s, %.0f GB/s (%.0f B per rating)\n",
                            mode, ms, n / ms / 1e6, n * bytes[mode] / ms / 1e6, bytes[mode]);
        }
    }
    return 0;
}
