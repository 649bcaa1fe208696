// mml_device.h -- device-side helpers shared by the .hip sources (never included by host-only
// .cpp files).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mml {

// Raw buffer resource over [base, base + bytes) (bytes < 2^32); dword 3 = the gfx9 raw-buffer
// format word.  Out-of-range offsets read 0 and drop stores.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

// Loads with the sc1 cache bit (aux bit 4): served by the XCD's L2, never by the CU's vector L1,
// which another CU's stores do not refresh (MI355X_MICROARCH.md, inter-workgroup visibility:
// "sc1 loads bypass L1 only, L2-served, 0-3 % slower than plain at 16 B").  For rows that only
// CUs of ONE XCD write (the XCD-owned item groups below) this is the load that sees every
// completed update.
__device__ __forceinline__ float4 load4_l2(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}
__device__ __forceinline__ float load1_l2(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 16));
}

// Stream spans of the XCD-owned item groups: group g's entries are [off[g], off[g + 1]).  Block b
// serves group b % ng (blocks b and b + 8 share an XCD, probed by
// mml::xcd_groups), so each group's rows are only ever cached in one XCD's L2.  ng = 1: one span,
// any block.
struct GroupWave {
    int64_t begin, end;
};
__device__ __forceinline__ GroupWave group_wave(const int64_t* __restrict__ goff, int32_t ng,
                                                int32_t waves_per_group, int wave_in_block,
                                                int waves_per_block) {
    const int g = (int)(blockIdx.x % (uint32_t)ng);
    const int64_t w = (int64_t)(blockIdx.x / (uint32_t)ng) * waves_per_block + wave_in_block;
    const int64_t g0 = goff[g], g1 = goff[g + 1];
    const int64_t chunk = (g1 - g0 + waves_per_group - 1) / waves_per_group;
    const int64_t b = min(g0 + w * chunk, g1);
    return GroupWave{b, min(b + chunk, g1)};
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64's finaliser
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// N(0, 1) draw number e of a counter-based stream keyed by seed (Box-Muller on two 53-bit
// uniforms): the device InitModel for models too large for the host RNG chain
__device__ __forceinline__ double counter_normal(uint64_t seed, uint64_t e) {
    const uint64_t x = mix64(seed ^ e * 0x9E3779B97F4A7C15ull);
    const double u1 = ((x >> 11) + 1.0) * (1.0 / 9007199254740993.0);  // (0, 1]
    const double u2 = (double)(mix64(x) >> 11) * (1.0 / 9007199254740992.0);
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

}  // namespace mml
