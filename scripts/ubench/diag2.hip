// Microbenchmark + check of wrmf_tiles.hip's diag_factor_mfma: T = L^{-1} of an SPD 32 x 32 tile
// held in the v_mfma_f32_32x32x2_f32 C/D layout, by column pairs on the matrix core.  Prints the
// cycles per factorisation (one wave, repeated) and max |T A T^T - I| against the input tile.
// hipcc --offload-arch=gfx950 -O3 diag2.hip -o diag2 -mllvm -amdgpu-mfma-vgpr-form=1 (as in the
// solve kernel, whose accumulators are VGPRs: AGPR accumulators add 2 x 16 moves per MFMA here)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr int kTS = 33;
__device__ __forceinline__ int rho(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }
__device__ __forceinline__ int opaque_tid() { int t = threadIdx.x; asm volatile("" : "+v"(t)); return t; }
__device__ __forceinline__ float lane_bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ float half_swap(float x, int h) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(h ? r[0] : r[1]);
}
__device__ __forceinline__ void diag_factor_mfma(f32x16 a, float (*tT)[kTS]) {
    const int lane = opaque_tid() & 63, q = lane & 31, h = lane >> 5;
    f32x16 r;
#pragma unroll
    for (int g = 0; g < 16; ++g) r[g] = rho(g, h) == q ? 1.0f : 0.0f;
#pragma unroll
    for (int c = 0; c < 32; c += 2) {
        const int hc = (c >> 2) & 1, gc = (c & 3) + 4 * (c >> 3);
        const float s0 = half_swap(a[gc], h), s1 = half_swap(a[gc + 1], h);
        const float a0 = h == hc ? a[gc] : s0;
        const float piv0 = lane_bcast(a0, c);
        const float rs0 = __builtin_amdgcn_rsqf(piv0);
        const float l0 = q < c ? 0.0f : (q == c ? piv0 * rs0 : a0 * rs0);
        const float l10 = lane_bcast(l0, c + 1);
        const float a1 = (h == hc ? a[gc + 1] : s1) - l0 * l10;
        const float piv1 = lane_bcast(a1, c + 1);
        const float rs1 = __builtin_amdgcn_rsqf(piv1);
        const float l1 = q <= c ? 0.0f : (q == c + 1 ? piv1 * rs1 : a1 * rs1);
        const float r0 = r[gc] * rs0;
        const float r1 = (r[gc + 1] - l10 * r0) * rs1;
        r[gc] = h == hc ? r0 : r[gc];
        r[gc + 1] = h == hc ? r1 : r[gc + 1];
        if (c + 2 < 32) {
            const float op = h ? l1 : l0;
            a = __builtin_amdgcn_mfma_f32_32x32x2f32(-op, op, a, 0, 0, 0);
            const float t0 = half_swap(r[gc], h), t1 = half_swap(r[gc + 1], h);
            const float opb = hc == 0 ? (h == 0 ? r[gc] : t1) : (h == 0 ? t0 : r[gc + 1]);
            const float opa = q > c + 1 ? op : 0.0f;
            r = __builtin_amdgcn_mfma_f32_32x32x2f32(-opa, opb, r, 0, 0, 0);
        }
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) tT[q][rho(g, h)] = r[g];
}
__global__ __launch_bounds__(64) void k(const float* A, float* out, long long* cyc, int reps) {
    __shared__ float tT[32][kTS];
    const int lane = threadIdx.x, q = lane & 31, h = lane >> 5;
    f32x16 a;
    for (int g = 0; g < 16; ++g) a[g] = A[q * 32 + rho(g, h)];
    long long t0 = clock64();
    for (int r = 0; r < reps; ++r) {
        diag_factor_mfma(a, tT);
        __builtin_amdgcn_s_barrier();
        a[0] += 0.0f * tT[q][0];
    }
    long long t1 = clock64();
    if (lane < 32) for (int m = 0; m < 32; ++m) out[lane * 32 + m] = tT[lane][m];  // tT[c][m] = T[m][c]
    if (lane == 0) cyc[0] = (t1 - t0) / reps;
}
int main() {
    const int n = 32;
    std::vector<float> A(n * n);
    // SPD: M M^T / n + d I with a spread of scales (condition ~1e4)
    std::vector<double> M(n * n);
    unsigned s = 1;
    for (auto& x : M) { s = s * 1103515245u + 12345u; x = ((s >> 8) & 0xFFFF) / 65536.0 - 0.5; }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v = 0;
            for (int t = 0; t < n; ++t) v += M[i * n + t] * M[j * n + t];
            A[i * n + j] = (float)(v + (i == j ? 1e-3 : 0.0));
        }
    float *dA, *dO; long long* dC;
    hipMalloc(&dA, sizeof(float) * n * n); hipMalloc(&dO, sizeof(float) * n * n); hipMalloc(&dC, 8);
    hipMemcpy(dA, A.data(), sizeof(float) * n * n, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dA, dO, dC, 1000);
    std::vector<float> T(n * n); long long cyc;
    hipMemcpy(T.data(), dO, sizeof(float) * n * n, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dC, 8, hipMemcpyDeviceToHost);
    // T[m][c] = out[c * 32 + m]; check T A T^T = I
    double err = 0, upper = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v = 0;
            for (int a_ = 0; a_ < n; ++a_)
                for (int b = 0; b < n; ++b) v += (double)T[a_ * n + i] * A[a_ * n + b] * T[b * n + j];
            err = std::fmax(err, std::fabs(v - (i == j ? 1.0 : 0.0)));
            if (j > i) upper = std::fmax(upper, std::fabs(T[i * n + j]));  // T[j][i], j > i: above diag
        }
    printf("diag_factor_mfma: %lld cycles per tile, max |T A T^T - I| = %.3g, max |upper| = %.3g\n",
           cyc, err, upper);
    return err < 1e-2 ? 0 : 1;
}
