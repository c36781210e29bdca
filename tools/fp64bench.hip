// VALU issue-price calibration by instruction class, for the `valu_issue` roof of bench.py (DESIGN.md
// section 3.2 and section 9.1).
//
// Round 5 measured FP64 add/mul/fma and an int32 add/xor chain (every one ~4 SIMD-cycles per wave64
// instruction).  The trajectory kernels also issue compares, selects, moves, FP64 division fix-ups,
// transcendental seeds, conversions and 64-bit integer ops (≈295 of the tiled Euler kernel's 1152 VALU
// instructions per wave-step were in no SQ_INSTS_VALU_* class), so round 6 prices each class alone.
//
// Every kernel runs 8 independent chains of ONE instruction per lane at 16 waves per SIMD (so no
// dependency stall is exposed and the SIMDs only issue that instruction).  The instruction is written as
// inline asm, so the count per wave is exact: kIters x kChains per wave (plus a few setup instructions,
// which the PMC pass sees and the time-only price ignores).  Each kernel prints one JSON object:
// wave64 instructions, hipEvent time, rate; the rocprofv3 pass over the same binary (tools/fp64bench.sh)
// gives GRBM_GUI_ACTIVE, so SIMD-cycles per wave instruction = (GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs
// / wave instructions, with SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_VALU2 beside it.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/fp64bench tools/fp64bench.hip
//
// Only vector (VGPR-destination or VALU-to-SGPR) instructions are timed here; nothing stores through
// the scalar data cache.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

constexpr int kChains = 8;
constexpr int kIters = 2048;

struct Args {
    const double* kd;      // [4] doubles
    const uint32_t* ku;    // [4] words
    uint64_t mask;         // a lane mask for v_cndmask (uniform, from the kernel argument: an SGPR pair)
    double* out;
};

// One op = one inline-asm instruction on chain j's register (v: double, f: float, u: u32, w: u64).
// The state is kept in all four types so one kernel template serves every class; only the type the
// op touches is live in the loop.
struct St {
    double v[kChains];
    float f[kChains];
    uint32_t u[kChains];
    uint64_t w[kChains];
    uint64_t m[kChains];  // lane masks written by compares / div_scale (one SGPR pair per chain)
    uint32_t r[kChains];  // readfirstlane results (one SGPR per chain)
};

#define OP(NAME, BODY)                                                                              \
    struct NAME {                                                                                   \
        static constexpr const char* name = #NAME;                                                  \
        __device__ __forceinline__ static void step(St& s, int j, double a, double b, uint32_t c,   \
                                                     uint32_t d, uint64_t m) {                      \
            (void)a; (void)b; (void)c; (void)d; (void)m;                                            \
            BODY;                                                                                   \
        }                                                                                           \
    };

// FP64 arithmetic (the classes SQ_INSTS_VALU_{FMA,ADD,MUL}_F64 count)
OP(fma_f64, asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(s.v[j]) : "v"(a), "v"(b)))
OP(add_f64, asm volatile("v_add_f64 %0, %0, %1" : "+v"(s.v[j]) : "v"(a)))
OP(mul_f64, asm volatile("v_mul_f64 %0, %0, %1" : "+v"(s.v[j]) : "v"(a)))
OP(max_f64, asm volatile("v_max_f64 %0, %0, %1" : "+v"(s.v[j]) : "v"(a)))
// FP64 division / sqrt expansion pieces (div_scale, div_fmas, div_fixup, ldexp, frexp, class)
OP(div_scale_f64, asm volatile("v_div_scale_f64 %0, %1, %0, %0, %2" : "+v"(s.v[j]), "+s"(s.m[j]) : "v"(a)))
OP(div_fmas_f64, asm volatile("v_div_fmas_f64 %0, %0, %1, %2" : "+v"(s.v[j]) : "v"(a), "v"(b)))
OP(div_fixup_f64, asm volatile("v_div_fixup_f64 %0, %0, %1, %2" : "+v"(s.v[j]) : "v"(a), "v"(b)))
OP(ldexp_f64, asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(s.v[j]) : "v"(c)))
OP(frexp_mant_f64, asm volatile("v_frexp_mant_f64 %0, %0" : "+v"(s.v[j])))
OP(cmp_class_f64, asm volatile("v_cmp_class_f64_e64 %0, %1, %2" : "+s"(s.m[j]) : "v"(s.v[j]), "v"(c)))
// FP64 transcendental seeds (SQ_INSTS_VALU_TRANS_F64)
OP(rcp_f64, asm volatile("v_rcp_f64 %0, %0" : "+v"(s.v[j])))
OP(rsq_f64, asm volatile("v_rsq_f64 %0, %0" : "+v"(s.v[j])))
OP(sqrt_f64, asm volatile("v_sqrt_f64 %0, %0" : "+v"(s.v[j])))
// compares writing a lane mask (SGPR pair), f64 and i32
OP(cmp_lt_f64, asm volatile("v_cmp_lt_f64_e64 %0, %1, %2" : "+s"(s.m[j]) : "v"(s.v[j]), "v"(a)))
OP(cmp_lt_i32, asm volatile("v_cmp_lt_i32_e64 %0, %1, %2" : "+s"(s.m[j]) : "v"(s.u[j]), "v"(c)))
// conversions (SQ_INSTS_VALU_CVT)
OP(cvt_f64_i32, asm volatile("v_cvt_f64_i32 %0, %1" : "+v"(s.v[j]) : "v"(s.u[j])))
OP(cvt_f32_f64, asm volatile("v_cvt_f32_f64 %0, %1" : "+v"(s.f[j]) : "v"(s.v[j])))
// 32-bit moves and selects
OP(mov_b32, asm volatile("v_mov_b32 %0, %1" : "+v"(s.u[j]) : "v"(c)))
OP(mov_b64, asm volatile("v_mov_b64 %0, %1" : "+v"(s.w[j]) : "v"(s.w[(j + 1) % kChains])))
OP(cndmask_b32, asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(s.u[j]) : "v"(d), "s"(m)))
OP(readfirstlane_b32, asm volatile("v_readfirstlane_b32 %0, %1" : "+s"(s.r[j]) : "v"(s.u[j])))
// 32-bit integer ALU (SQ_INSTS_VALU_INT32)
OP(add_u32, asm volatile("v_add_u32 %0, %0, %1" : "+v"(s.u[j]) : "v"(c)))
OP(xor_b32, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(s.u[j]) : "v"(c)))
OP(mul_lo_u32, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(s.u[j]) : "v"(c)))
OP(lshl_add_u32, asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(s.u[j]) : "v"(c)))
// 64-bit integer (SQ_INSTS_VALU_INT64) and the address forms the compiler emits
OP(lshlrev_b64, asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(s.w[j])))
OP(lshl_add_u64, asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(s.w[j]) : "v"(s.w[(j + 3) % kChains])))
OP(mad_u64_u32, asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(s.w[j]), "+s"(s.m[j]) : "v"(c), "v"(d)))
// FP32 (the guide's SIMD-32 rows: v_fma_f32 2 cycles wave64) and packed FP32
OP(fma_f32, asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s.f[j]) : "v"((float)a), "v"((float)b)))
OP(add_f32, asm volatile("v_add_f32 %0, %0, %1" : "+v"(s.f[j]) : "v"((float)a)))
OP(pk_fma_f32, asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(s.w[j]) : "v"(s.w[(j + 2) % kChains]), "v"(s.w[(j + 5) % kChains])))
OP(rcp_f32, asm volatile("v_rcp_f32 %0, %0" : "+v"(s.f[j])))

template <class Op>
__global__ void __launch_bounds__(256) fb_kernel(Args g) {
    const double a = g.kd[0], b = g.kd[1];
    const uint32_t c = g.ku[0], d = g.ku[1];
    St s;
#pragma unroll
    for (int j = 0; j < kChains; ++j) {
        s.v[j] = g.kd[2] + j + threadIdx.x;
        s.f[j] = (float)s.v[j];
        s.u[j] = g.ku[2] + j + threadIdx.x;
        s.w[j] = ((uint64_t)s.u[j] << 20) | j;
        s.m[j] = 0;
        s.r[j] = 0;
    }
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < kChains; ++j) Op::step(s, j, a, b, c, d, g.mask);
    }
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < kChains; ++j) acc += s.v[j] + s.f[j] + (double)s.u[j] + (double)(s.w[j] & 0xffff) + (double)(s.m[j] & 0xff) + s.r[j];
    g.out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

struct Entry {
    const char* name;
    void (*fn)(Args);
    const char* cls;  // the SQ_INSTS_VALU_* class the instruction is counted in (by the ISA manual)
};

#define E(NAME, CLS) {NAME::name, fb_kernel<NAME>, CLS}
static const Entry kEntries[] = {
    E(fma_f64, "FMA_F64"),       E(add_f64, "ADD_F64"),        E(mul_f64, "MUL_F64"),
    E(max_f64, "?"),             E(div_scale_f64, "?"),        E(div_fmas_f64, "?"),
    E(div_fixup_f64, "?"),       E(ldexp_f64, "?"),            E(frexp_mant_f64, "?"),
    E(cmp_class_f64, "?"),       E(rcp_f64, "TRANS_F64"),      E(rsq_f64, "TRANS_F64"),
    E(sqrt_f64, "TRANS_F64"),    E(cmp_lt_f64, "?"),           E(cmp_lt_i32, "?"),
    E(cvt_f64_i32, "CVT"),       E(cvt_f32_f64, "CVT"),        E(mov_b32, "?"),
    E(mov_b64, "?"),             E(cndmask_b32, "?"),          E(readfirstlane_b32, "?"),
    E(add_u32, "INT32"),         E(xor_b32, "INT32"),          E(mul_lo_u32, "INT32"),
    E(lshl_add_u32, "INT32"),    E(lshlrev_b64, "INT64"),      E(lshl_add_u64, "INT64"),
    E(mad_u64_u32, "INT64"),     E(fma_f32, "FMA_F32"),        E(add_f32, "ADD_F32"),
    E(pk_fma_f32, "FMA_F32"),    E(rcp_f32, "TRANS_F32"),
};

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    const char* only = argc > 2 ? argv[2] : nullptr;  // run one kernel by name
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 16;  // 64 waves per CU = 16 per SIMD
    const int threads = 256;
    const int64_t n = (int64_t)blocks * threads;
    Args g{};
    double* dk;
    uint32_t* uk;
    CK(hipMalloc(&dk, 4 * sizeof(double)));
    CK(hipMalloc(&uk, 4 * sizeof(uint32_t)));
    CK(hipMalloc(&g.out, n * sizeof(double)));
    const double hk[4] = {0.9999999, 1e-9, 1.0, 0.0};
    const uint32_t hu[4] = {3u, 0x7F4A7C15u, 1u, 0u};
    CK(hipMemcpy(dk, hk, sizeof(hk), hipMemcpyHostToDevice));
    CK(hipMemcpy(uk, hu, sizeof(hu), hipMemcpyHostToDevice));
    g.kd = dk;
    g.ku = uk;
    g.mask = 0x5555555555555555ull;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double waves = (double)blocks * (threads / 64);
    const double insts = waves * kIters * kChains;
    for (const Entry& e : kEntries) {
        if (only && strcmp(only, e.name) != 0) continue;
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(e.fn, dim3(blocks), dim3(threads), 0, 0, g);
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        printf("{\"kernel\": \"%s\", \"class\": \"%s\", \"wave_insts\": %.6e, \"ms\": %.4f, "
               "\"wave_insts_per_s\": %.6e, \"cus\": %d}\n",
               e.name, e.cls, insts, best, insts / (best * 1e-3), prop.multiProcessorCount);
        fflush(stdout);
    }
    CK(hipFree(dk));
    CK(hipFree(uk));
    CK(hipFree(g.out));
    return 0;
}
