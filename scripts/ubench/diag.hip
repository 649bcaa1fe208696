// Microbenchmark: cycles of the 32x32 diagonal factorisation + inverse used by wrmf_tiles.hip
// (one wave per workgroup, repeated on an SPD tile in LDS).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(fast)
__device__ __forceinline__ float lane_bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ int opaque(int t) { asm volatile("" : "+v"(t)); return t; }
template <int MODE>
__global__ __launch_bounds__(64) void k_diag(float* out, long long* cyc, int reps) {
    __shared__ float dg[32][36];
    __shared__ float tT[32][40];
    const int lane = opaque(threadIdx.x), q = lane & 31, h = lane >> 5;
    for (int c = 0; c < 32; ++c) dg[q][c] = (q == c ? 40.0f : 0.0f) + 1.0f / (1 + q + c);
    __syncthreads();
    long long t0 = clock64();
    float keep = 0.f;
    for (int r = 0; r < reps; ++r) {
        float x[32];
#pragma unroll
        for (int c = 0; c < 32; c += 4) {
            const float4 v = *reinterpret_cast<const float4*>(&dg[q][c]);
            x[c] = v.x; x[c + 1] = v.y; x[c + 2] = v.z; x[c + 3] = v.w;
        }
        if (MODE & 1) {
#pragma unroll
            for (int c = 0; c < 32; ++c) {
                const float piv = lane_bcast(x[c], c);
                const float inv = __builtin_amdgcn_rsqf(piv);
                x[c] = (q == c) ? piv * inv : x[c] * inv;
#pragma unroll
                for (int c2 = c + 1; c2 < 32; ++c2) x[c2] -= x[c] * lane_bcast(x[c], c2);
            }
        }
        if (MODE & 4) {
            typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int c = 0; c < 32; ++c) {
                const float piv = lane_bcast(x[c], c);
                const float inv = __builtin_amdgcn_rsqf(piv);
                x[c] = (q == c) ? piv * inv : x[c] * inv;
                const f2 xc = {x[c], x[c]};
#pragma unroll
                for (int c2 = c + 1; c2 < 32; c2 += 2) {
                    if (c2 + 1 < 32) {
                        f2 a = {x[c2], x[c2 + 1]};
                        const f2 l = {lane_bcast(x[c], c2), lane_bcast(x[c], c2 + 1)};
                        a = a - xc * l;
                        x[c2] = a.x; x[c2 + 1] = a.y;
                    } else {
                        x[c2] -= x[c] * lane_bcast(x[c], c2);
                    }
                }
            }
        }
        if (MODE & 2) {
            float tc[32];
#pragma unroll
            for (int m = 0; m < 32; ++m) {
                float s0 = (m == q) ? 1.0f : 0.0f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
                for (int j4 = 0; j4 < m; j4 += 4) {
                    const float4 l = *reinterpret_cast<const float4*>(&dg[m][j4]);
                    s0 -= l.x * tc[j4];
                    if (j4 + 1 < m) s1 -= l.y * tc[j4 + 1];
                    if (j4 + 2 < m) s2 -= l.z * tc[j4 + 2];
                    if (j4 + 3 < m) s3 -= l.w * tc[j4 + 3];
                }
                tc[m] = ((s0 + s1) + (s2 + s3)) * __builtin_amdgcn_rcpf(dg[m][m]);
            }
            if (h == 0)
#pragma unroll
                for (int m = 0; m < 32; ++m) tT[q][m] = tc[m];
            keep += tT[q][q & 7];
        }
        if (MODE & 8) {  // right-looking inverse: column j of L from a transposed copy in LDS
            __shared__ float lT[32][36];
            if (h == 0)
#pragma unroll
                for (int c = 0; c < 32; ++c) lT[c][q] = x[c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            float sv[32];
#pragma unroll
            for (int m = 0; m < 32; ++m) sv[m] = (m == q) ? 1.0f : 0.0f;
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                sv[j] *= __builtin_amdgcn_rcpf(lT[j][j]);
#pragma unroll
                for (int m4 = (j + 1) & ~3; m4 < 32; m4 += 4) {
                    const float4 l = *reinterpret_cast<const float4*>(&lT[j][m4]);
                    if (m4 > j) sv[m4] -= l.x * sv[j];
                    if (m4 + 1 > j) sv[m4 + 1] -= l.y * sv[j];
                    if (m4 + 2 > j) sv[m4 + 2] -= l.z * sv[j];
                    if (m4 + 3 > j) sv[m4 + 3] -= l.w * sv[j];
                }
            }
            if (h == 0)
#pragma unroll
                for (int m = 0; m < 32; ++m) tT[q][m] = sv[m];
            keep += tT[q][q & 7];
        }
        if (MODE & 16) {  // the kernel's single-accumulator inverse
            float tc[32];
#pragma unroll
            for (int m = 0; m < 32; ++m) {
                float sacc = (m == q) ? 1.0f : 0.0f;
#pragma unroll
                for (int j4 = 0; j4 < m; j4 += 4) {
                    const float4 l = *reinterpret_cast<const float4*>(&dg[m][j4]);
                    sacc -= l.x * tc[j4];
                    if (j4 + 1 < m) sacc -= l.y * tc[j4 + 1];
                    if (j4 + 2 < m) sacc -= l.z * tc[j4 + 2];
                    if (j4 + 3 < m) sacc -= l.w * tc[j4 + 3];
                }
                tc[m] = sacc * __builtin_amdgcn_rcpf(dg[m][m]);
            }
            if (h == 0)
#pragma unroll
                for (int m = 0; m < 32; ++m) tT[q][m] = tc[m];
            keep += tT[q][q & 7];
        }
#pragma unroll
        for (int c = 0; c < 32; ++c) keep += x[c];
        asm volatile("" : "+v"(keep));
    }
    long long t1 = clock64();
    out[blockIdx.x * 64 + lane] = keep;
    if (lane == 0) cyc[blockIdx.x] = (t1 - t0) / reps;
}
int main() {
    float* out; long long* cyc;
    hipMalloc(&out, 256 * 64 * 4); hipMalloc(&cyc, 256 * 8);
    long long h[256];
    auto run = [&](auto kern, const char* name) {
        kern<<<256, 64>>>(out, cyc, 200);
        hipDeviceSynchronize();
        kern<<<256, 64>>>(out, cyc, 200);
        hipMemcpy(h, cyc, 256 * 8, hipMemcpyDeviceToHost);
        printf("%-20s %lld cycles per call (clock64)\n", name, h[0]);
    };
    run(k_diag<0>, "load only");
    run(k_diag<1>, "factor");
    run(k_diag<2>, "inverse");
    run(k_diag<3>, "factor+inverse");
    run(k_diag<4>, "factor packed");
    run(k_diag<6>, "packed+inverse");
    run(k_diag<16>, "inverse 1-acc");
    run(k_diag<8>, "inverse right");
    run(k_diag<17>, "factor+inv 1-acc");
    run(k_diag<9>, "factor+inv right");
    return 0;
}
