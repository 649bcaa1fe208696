// Checks the planes Gram's operand reads (wrmf_tiles.hip gram_accumulate_p3) on the device: a
// vector-major LDS image of 16 vectors x 256 bf16 (16-B chunk ch of vector v at position
// ch ^ ((v & 3) << 2)), read with ds_read_b64_tr_b16 as the 32x32x16 MFMA operand of feature
// block X: lane (q, h) must get vectors 8h .. 8h + 7 of feature 32 X + q.  Prints mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
using v4s = __attribute__((ext_vector_type(4))) short;
__device__ __forceinline__ v4s lds_tr16(const uint16_t* p) {
    using lp = __attribute__((address_space(3))) v4s*;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(__attribute__((address_space(3))) void*)(p));
}
__global__ void k(int* bad, short* out) {
    __shared__ __attribute__((aligned(16))) uint16_t img[16][256];
    const int lane = threadIdx.x;
    for (int x = lane; x < 16 * 256; x += 64) {  // value = v * 256 + f at its swizzled position
        const int v = x / 256, f = x % 256;
        const int ch = f / 8, pos = ch ^ ((v & 3) << 2);
        img[v][pos * 8 + f % 8] = (uint16_t)(v * 256 + f);
    }
    __syncthreads();
    const int g4 = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3, q = lane & 31, h = lane >> 5;
    const int rowv = 8 * (g4 >> 1) + qq;
    for (int X = 0; X < 8; ++X) {
        const int ch = 4 * X + 2 * (g4 & 1) + (pp >> 1);
        const uint16_t* a0 = &img[rowv][8 * (ch ^ (qq << 2)) + 4 * (pp & 1)];
        const v4s lo = lds_tr16(a0), hi = lds_tr16(a0 + 4 * 256);
        const short e[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        for (int j = 0; j < 8; ++j) {
            const int want = (8 * h + j) * 256 + 32 * X + q;
            if ((uint16_t)e[j] != want) atomicAdd(bad, 1);
            if (X == 1) out[lane * 8 + j] = e[j];
        }
    }
}
int main() {
    int* bad; short* out;
    hipMalloc(&bad, 4); hipMemset(bad, 0, 4); hipMalloc(&out, 64 * 8 * 2);
    k<<<1, 64>>>(bad, out);
    int h = -1; short o[512];
    hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
    hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
    printf("tr16 operand mismatches: %d of %d\n", h, 8 * 64 * 8);
    for (int l = 0; l < 64; l += 13) {
        printf("lane %2d:", l);
        for (int j = 0; j < 8; ++j) printf(" v%d f%d", (uint16_t)o[l * 8 + j] / 256, (uint16_t)o[l * 8 + j] % 256);
        printf("\n");
    }
    return h == 0 ? 0 : 1;
}
