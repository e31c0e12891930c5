// VALU issue prices on the whole chip, timed by HIP events (gfx950).  Resolves the round-4
// contradiction of valu_cost.hip (one workgroup, s_memtime around the loop: 4.2-4.4 cycles
// per plain wave64 instruction per SIMD at four waves per SIMD, against the 2 the issue model
// and MI355X_MICROARCH.md use).
//
// Grid: 256 x W workgroups of 256 threads (one wave per SIMD per workgroup, so W waves per
// SIMD when the dispatcher spreads them), every lane runs CHAINS independent chains of one
// instruction REPS times.  Per-SIMD cycles per wave-instruction =
//     (event_time(REPS) - event_time(REPS / 2)) * clock * 1024 SIMDs / (wave-instructions of the
//     difference)  -- the differential cancels launch ramp-up, tail and fixed per-wave work,
// quoted at the nominal 2.4 GHz and at the in-kernel clock (delta s_memtime / delta
// s_memrealtime x 100 MHz, median over workgroups).  A one-workgroup run (the old probe's
// shape) reports the same two clocks, which shows what its s_memtime cycles were.
//   hipcc -O3 --offload-arch=gfx950 scripts/diag/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHAINS 8

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t *out, uint64_t *stamp, uint32_t seed, int reps) {
    uint32_t x[CHAINS];
    uint64_t p[CHAINS], q[CHAINS];
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) {
        x[i] = seed * (threadIdx.x + 17 * i) + i;
        p[i] = (uint64_t)x[i] * 0x9E3779B97F4A7C15ull;
        q[i] = 0x3F8000013F800001ull ^ ((uint64_t)i << 3);
    }
    const uint32_t K = 0x3F800001u ^ seed;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int i = 0; i < CHAINS; ++i) {
                if constexpr (OP == 0) asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[i]) : "s"(K));
                if constexpr (OP == 1) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(x[i]) : "s"(K));
                if constexpr (OP == 2) {
                    uint64_t p = x[i] | ((uint64_t)x[i] << 32);
                    asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(p));
                    x[i] = (uint32_t)p;
                }
                if constexpr (OP == 3) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i]));
                if constexpr (OP == 4) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[i]) : "s"(K));
                if constexpr (OP == 5) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "s"(K));
                if constexpr (OP == 6) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(K));
                // packed f32 with distinct operand pairs (OP 2 reads one pair three times)
                if constexpr (OP == 7) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(q[i]));
                if constexpr (OP == 8) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(q[i]), "v"(q[(i + 1) % CHAINS]));
                if constexpr (OP == 9) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(q[i]));
                if constexpr (OP == 10) {  // one packed FMA + one plain add, independent
                    asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(q[i]), "v"(q[(i + 1) % CHAINS]));
                    asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[i]) : "s"(K));
                }
                if constexpr (OP == 11) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p[i]) : "v"(x[i]), "s"(K) : "vcc");
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) a ^= x[i] ^ (uint32_t)p[i] ^ (uint32_t)(p[i] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if (threadIdx.x == 0) {
        stamp[2 * blockIdx.x] = t1 - t0;
        stamp[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// instructions a step issues per chain (OP 10: a packed FMA and a plain add)
template <int OP> constexpr int instr_per_step() { return OP == 10 ? 2 : 1; }

// One timed series: 5 launches of `reps` repetitions after 3 warm-up launches; returns the event
// milliseconds of the 5 and fills the stamps of the last.
template <int OP>
float timed(uint32_t *out, uint64_t *stamp, int blocks, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) kern<OP><<<blocks, 256>>>(out, stamp, 1 + w, reps);  // warm the clock
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int l = 0; l < 5; ++l) kern<OP><<<blocks, 256>>>(out, stamp, 7 + l, reps);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms;
}

// Differential: the series at reps and at reps / 2, so launch ramp-up, tail and fixed per-wave
// cost cancel; wave-instructions = blocks x 4 waves x (reps - reps/2) x 4 unroll x CHAINS x
// instructions per step.
template <int OP>
void run(const char *name, int blocks, int reps, bool one_wg) {
    uint32_t *out;
    uint64_t *stamp;
    hipMalloc(&out, (size_t)4 * 256 * blocks);
    hipMalloc(&stamp, (size_t)16 * blocks);
    const int half = reps / 2;
    const float ms_half = timed<OP>(out, stamp, blocks, half);
    std::vector<uint64_t> hh((size_t)2 * blocks);
    hipMemcpy(hh.data(), stamp, (size_t)16 * blocks, hipMemcpyDeviceToHost);
    const float ms = timed<OP>(out, stamp, blocks, reps);
    std::vector<uint64_t> h((size_t)2 * blocks);
    hipMemcpy(h.data(), stamp, (size_t)16 * blocks, hipMemcpyDeviceToHost);
    std::vector<double> clk(blocks), dcyc(blocks);
    for (int i = 0; i < blocks; ++i) {
        clk[i] = (double)h[2 * i] / (double)h[2 * i + 1] * 0.1;  // GHz: memtime ticks per 100 MHz tick
        dcyc[i] = (double)h[2 * i] - (double)hh[2 * i];
    }
    std::sort(clk.begin(), clk.end());
    std::sort(dcyc.begin(), dcyc.end());
    const double ghz = clk[blocks / 2];
    const double per_wave = (double)(reps - half) * 4 * CHAINS * instr_per_step<OP>();  // per wave, differential
    const double ds = (ms - ms_half) * 1e-3 / 5;  // seconds per launch, differential
    if (one_wg) {
        // one workgroup = one wave per SIMD on one CU: cycles per wave-instruction of ONE wave
        printf("{\"op\": \"%s\", \"shape\": \"1 workgroup, 1 wave/SIMD\", \"memtime_ghz\": %.3f, "
               "\"memtime_cycles_per_wave_instr\": %.3f, \"event_cycles_per_wave_instr_at_2.4GHz\": %.3f}\n",
               name, ghz, dcyc[blocks / 2] / per_wave, ds * 2.4e9 / per_wave);
    } else {
        const int W = blocks / 256;
        const double wave_instr = (double)blocks * 4 * per_wave;
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms_per_launch\": %.4f, \"memtime_ghz\": %.3f, "
               "\"simd_cycles_per_wave_instr_at_2.4GHz\": %.3f, \"simd_cycles_per_wave_instr_at_memtime_clock\": %.3f, "
               "\"method\": \"differential: (t(reps) - t(reps/2)), 5 launches each\"}\n",
               name, W, ms / 5, ghz, ds * 2.4e9 * 1024 / wave_instr, ds * ghz * 1e9 * 1024 / wave_instr);
    }
    fflush(stdout);
    hipFree(out);
    hipFree(stamp);
}

template <int OP>
void sweep(const char *name) {
    run<OP>(name, 1, 1 << 14, true);
    for (int W : {1, 2, 4, 8}) run<OP>(name, 256 * W, 1 << 12, false);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
    sweep<0>("v_add_f32");
    sweep<1>("v_fma_f32");
    sweep<2>("v_pk_mul_f32");
    sweep<3>("v_rcp_f32");
    sweep<4>("v_xor_b32");
    sweep<5>("v_mul_lo_u32");
    sweep<6>("v_cndmask_b32");
    sweep<7>("v_pk_mul_f32 distinct");
    sweep<8>("v_pk_fma_f32 distinct");
    sweep<9>("v_pk_add_f32 distinct");
    sweep<10>("v_pk_fma_f32 + v_add_f32 (2 instr)");
    sweep<11>("v_mad_u64_u32");
    return 0;
}
