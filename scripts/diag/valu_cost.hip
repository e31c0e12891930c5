// Issue cost of the integer VALU instructions the graph sampler's Philox rounds use (gfx950).
// One workgroup; each lane runs 8 independent chains of one instruction, 256 times; cycles per
// wave-instruction from s_memtime around the loop (shader clock).  Waves per SIMD = blockDim/256
// when blockDim >= 256 (64: one wave on one SIMD).
//   hipcc -O3 --offload-arch=gfx950 scripts/diag/valu_cost.hip -o /tmp/valu_cost && /tmp/valu_cost
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define REPS 256

template <int OP>
__global__ void kern(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t x[CHAINS];
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) x[i] = seed * (threadIdx.x + 17 * i) + i;
    const uint32_t K = 0xD2511F53u;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int i = 0; i < CHAINS; ++i) {
            if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 2) {
                uint64_t p, c;
                asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(c) : "v"(x[i]), "s"(K));
                x[i] = (uint32_t)p ^ (uint32_t)(p >> 32);
            }
            if constexpr (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 4) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 5) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 6) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 8) asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 9) {
                uint64_t p = x[i] | ((uint64_t)x[i] << 32);
                asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(p));
                x[i] = (uint32_t)p;
            }
            if constexpr (OP == 10) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i]));
            if constexpr (OP == 11) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(K ^ x[i]));
            if constexpr (OP == 12) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
            if constexpr (OP == 13) asm volatile("v_med3_f32 %0, %0, %1, %0" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 14) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 15) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 16) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x[i]) : "s"(K));
            if constexpr (OP == 7) {  // mad_u64 alone (result kept, no xor)
                uint64_t p, c;
                asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(c) : "v"(x[i]), "s"(K));
                x[i] = (uint32_t)(p >> 32);
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) a ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

template <int OP>
void run(const char *name, int threads) {
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, 4 * 1024);
    hipMalloc(&cyc, 8 * 16);
    kern<OP><<<1, threads>>>(out, cyc, 1);
    hipDeviceSynchronize();
    kern<OP><<<1, threads>>>(out, cyc, 3);
    hipDeviceSynchronize();
    uint64_t h[16];
    hipMemcpy(h, cyc, 8 * 16, hipMemcpyDeviceToHost);
    const int waves = threads / 64;
    uint64_t mx = 0;
    for (int w = 0; w < waves; ++w) mx = h[w] > mx ? h[w] : mx;
    const double per = (double)mx / (REPS * CHAINS);
    printf("%-26s threads %4d waves/SIMD %d : %6.2f cycles per wave-instruction (per SIMD: %6.2f)\n", name, threads,
           waves >= 4 ? waves / 4 : 1, per, per / (waves >= 4 ? waves / 4 : 1));
    hipFree(out);
    hipFree(cyc);
}

// s_memtime ticks per second: a long single-wave loop timed by s_memtime and by HIP events
__global__ void spin(uint64_t *cyc, uint32_t n) {
    uint32_t x = threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "s"(i));
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = x; }
}

int main() {
    {
        uint64_t *cyc;
        hipMalloc(&cyc, 16);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        spin<<<1, 64>>>(cyc, 1000);
        hipDeviceSynchronize();
        hipEventRecord(a);
        spin<<<1, 64>>>(cyc, 20000000);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        uint64_t h[2];
        hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
        printf("s_memtime: %llu ticks in %.3f ms = %.3f GHz (loop of 2e7 v_xor: %.2f ticks per iteration)\n",
               (unsigned long long)h[0], ms, h[0] / (ms * 1e6), h[0] / 2e7);
    }
    for (int t : {64, 256, 512, 1024}) {
        run<0>("v_mul_lo_u32", t);
        run<1>("v_mul_hi_u32", t);
        run<2>("v_mad_u64_u32 (+xor)", t);
        run<7>("v_mad_u64_u32", t);
        run<3>("v_mul_u32_u24", t);
        run<5>("v_mul_hi_u32_u24", t);
        run<4>("v_xor_b32", t);
        run<6>("v_bitop3_b32 (xor3)", t);
        run<8>("v_add_f32", t);
        run<16>("v_mul_f32", t);
        run<14>("v_fma_f32", t);
        run<9>("v_pk_mul_f32", t);
        run<10>("v_rcp_f32", t);
        run<12>("v_exp_f32", t);
        run<13>("v_med3_f32", t);
        run<11>("v_cndmask_b32", t);
        run<15>("v_and_b32", t);
    }
    return 0;
}
