// FP64 VALU issue-rate microbenchmark for the `valu_issue` roof of bench.py.
//
// The roof prices a wave64 FP64 add / mul / fma at 4 SIMD-cycles and any other VALU instruction at 2,
// from the vendor's 78.6 TFLOP/s vector FP64 figure (MI355X_MICROARCH.md lists no FP64 rate).  These
// kernels measure it: each lane runs 8 independent chains of one FP64 operation (no dependency stalls
// at 16 waves per SIMD), so the SIMDs do nothing but issue that instruction.
//
//  fb_fma  v_fma_f64        fb_add  v_add_f64        fb_mul  v_mul_f64
//  fb_i32  v_add_u32 / v_xor_b32 (a 32-bit integer chain: the "other VALU" price)
//  fb_mix  2 FP64 fma + 1 int32 op per step (does other VALU work overlap FP64 issue?)
//
// Each kernel prints one JSON object: wave64 instructions, hipEvent time, and the rate; a rocprofv3
// pass with GRBM_GUI_ACTIVE over the same binary gives the cycles (tools/fp64bench.sh), so
// SIMD-cycles per wave instruction = (GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs / wave instructions.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/fp64bench tools/fp64bench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

constexpr int kChains = 8;
constexpr int kIters = 4096;

// the coefficients come from memory so nothing folds; the results go to memory so nothing is dead
__global__ void __launch_bounds__(256) fb_fma(const double* __restrict__ k, double* __restrict__ out) {
    const double a = k[0], b = k[1];
    double v[kChains];
#pragma unroll
    for (int j = 0; j < kChains; ++j) v[j] = k[2] + j + threadIdx.x;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < kChains; ++j) v[j] = __builtin_fma(v[j], a, b);
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < kChains; ++j) s += v[j];
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) fb_add(const double* __restrict__ k, double* __restrict__ out) {
    const double a = k[0];
    double v[kChains];
#pragma unroll
    for (int j = 0; j < kChains; ++j) v[j] = k[2] + j + threadIdx.x;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < kChains; ++j) v[j] = v[j] + a;
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < kChains; ++j) s += v[j];
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) fb_mul(const double* __restrict__ k, double* __restrict__ out) {
    const double a = k[0];
    double v[kChains];
#pragma unroll
    for (int j = 0; j < kChains; ++j) v[j] = k[2] + j + threadIdx.x;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < kChains; ++j) v[j] = v[j] * a;
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < kChains; ++j) s += v[j];
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) fb_i32(const uint32_t* __restrict__ k, uint32_t* __restrict__ out) {
    const uint32_t a = k[0], b = k[1];
    uint32_t v[kChains];
#pragma unroll
    for (int j = 0; j < kChains; ++j) v[j] = k[2] + j + threadIdx.x;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < kChains; ++j) v[j] = (v[j] + a) ^ b;  // two VALU ops per chain step
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kChains; ++j) s += v[j];
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) fb_mix(const double* __restrict__ k, const uint32_t* __restrict__ ki,
                                              double* __restrict__ out) {
    const double a = k[0], b = k[1];
    const uint32_t c = ki[0], c2 = ki[1];
    double v[kChains];
    uint32_t u[kChains / 2];
#pragma unroll
    for (int j = 0; j < kChains; ++j) v[j] = k[2] + j + threadIdx.x;
#pragma unroll
    for (int j = 0; j < kChains / 2; ++j) u[j] = ki[2] + j + threadIdx.x;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < kChains; ++j) v[j] = __builtin_fma(v[j], a, b);
#pragma unroll
        for (int j = 0; j < kChains / 4; ++j) u[j] = (u[j] + c) ^ c2;  // 1 int op per 2 FP64 fma
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < kChains; ++j) s += v[j];
#pragma unroll
    for (int j = 0; j < kChains / 2; ++j) s += (double)u[j];
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 16;  // 64 waves per CU = 16 per SIMD
    const int threads = 256;
    const int64_t n = (int64_t)blocks * threads;
    double *dk, *dout;
    uint32_t *ik, *iout;
    CK(hipMalloc(&dk, 4 * sizeof(double)));
    CK(hipMalloc(&ik, 4 * sizeof(uint32_t)));
    CK(hipMalloc(&dout, n * sizeof(double)));
    CK(hipMalloc(&iout, n * sizeof(uint32_t)));
    const double hk[4] = {0.9999999, 1e-9, 1.0, 0.0};
    const uint32_t hik[4] = {0x9E3779B1u, 0x7F4A7C15u, 1u, 0u};
    CK(hipMemcpy(dk, hk, sizeof(hk), hipMemcpyHostToDevice));
    CK(hipMemcpy(ik, hik, sizeof(hik), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double waves = (double)blocks * (threads / 64);
    struct K {
        const char* name;
        double insts_per_step;  // wave64 instructions per chain step per wave (all chains)
        double flops_per_inst;  // per lane
        int kind;
    } ks[] = {{"fb_fma", kChains, 2.0, 0}, {"fb_add", kChains, 1.0, 1}, {"fb_mul", kChains, 1.0, 2},
              {"fb_i32", 2.0 * kChains, 0.0, 3}, {"fb_mix", kChains + kChains / 2, 0.0, 4}};
    for (const K& kk : ks) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            switch (kk.kind) {
                case 0: fb_fma<<<blocks, threads>>>(dk, dout); break;
                case 1: fb_add<<<blocks, threads>>>(dk, dout); break;
                case 2: fb_mul<<<blocks, threads>>>(dk, dout); break;
                case 3: fb_i32<<<blocks, threads>>>(ik, iout); break;
                default: fb_mix<<<blocks, threads>>>(dk, ik, dout); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        const double insts = waves * kIters * kk.insts_per_step;
        const double flops = insts * 64.0 * kk.flops_per_inst;
        printf("{\"kernel\": \"%s\", \"wave_insts\": %.6e, \"ms\": %.4f, \"wave_insts_per_s\": %.6e, "
               "\"tflops\": %.3f, \"cus\": %d}\n",
               kk.name, insts, best, insts / (best * 1e-3), flops / (best * 1e-3) / 1e12, prop.multiProcessorCount);
    }
    CK(hipFree(dk));
    CK(hipFree(ik));
    CK(hipFree(dout));
    CK(hipFree(iout));
    return 0;
}
