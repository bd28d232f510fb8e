// valu_rate.hip — measures issue throughput of the integer VALU instructions
// the digest kernels are built from (cycles per wave64 instruction per SIMD).
// Each thread runs 8 independent dependency chains of one instruction form in
// inline asm; 256 CUs x 8 waves/SIMD.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(X) X X X X X X X X
#define CHAINS(OP) \
    asm volatile(REP8(OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")) \
                 : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) \
                 : "v"(k0), "v"(k1));

#define OP_ADD(r) "v_add_u32 " r ", " r ", %8\n"
#define OP_ADD3(r) "v_add3_u32 " r ", " r ", %8, %9\n"
#define OP_ALIGNBIT(r) "v_alignbit_b32 " r ", " r ", %8, 7\n"
#define OP_BITOP3(r) "v_bitop3_b32 " r ", " r ", %8, %9 bitop3:0x96\n"
#define OP_XOR(r) "v_xor_b32 " r ", " r ", %8\n"
#define OP_PERM(r) "v_perm_b32 " r ", " r ", %8, %9\n"
#define OP_LSHLADD(r) "v_lshl_add_u32 " r ", " r ", 3, %8\n"
#define OP_BFE(r) "v_bfe_u32 " r ", " r ", 8, 8\n"
#define OP_XAD(r) "v_xad_u32 " r ", " r ", %8, %9\n"
#define OP_FMA(r) "v_fma_f32 " r ", " r ", %8, %9\n"
#define OP_SHL(r) "v_lshlrev_b32 " r ", 3, " r "\n"
#define OP_SHR(r) "v_lshrrev_b32 " r ", 3, " r "\n"
#define OP_LSHLOR(r) "v_lshl_or_b32 " r ", " r ", 3, %8\n"
#define OP_ALIGNBYTE(r) "v_alignbyte_b32 " r ", " r ", %8, 1\n"
#define OP_MOV(r) "v_mov_b32 " r ", " r "\n"
#define OP_BFI(r) "v_bfi_b32 " r ", " r ", %8, %9\n"
#define OP_OR3(r) "v_or3_b32 " r ", " r ", %8, %9\n"
#define OP_CNDMASK(r) "v_cndmask_b32 " r ", " r ", %8, vcc\n"
// Same VGPR read twice (a rotate is v_alignbit x, x, n).
#define OP_ALIGNBIT_SAME(r) "v_alignbit_b32 " r ", " r ", " r ", 7\n"
#define OP_PERM_SAME(r) "v_perm_b32 " r ", " r ", " r ", %9\n"
#define OP_XOR_SAME(r) "v_xor_b32 " r ", " r ", " r "\n"
#define OP_ADD_SAME(r) "v_add_u32 " r ", " r ", " r "\n"

#define KERNEL(NAME, OP)                                                             \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, int iters) {          \
        unsigned r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, \
                 r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;                              \
        unsigned k0 = blockIdx.x | 1, k1 = 0x01010101u;                              \
        for (int i = 0; i < iters; ++i) { CHAINS(OP) }                               \
        out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;  \
    }

KERNEL(k_add, OP_ADD)
KERNEL(k_add3, OP_ADD3)
KERNEL(k_alignbit, OP_ALIGNBIT)
KERNEL(k_bitop3, OP_BITOP3)
KERNEL(k_xor, OP_XOR)
KERNEL(k_perm, OP_PERM)
KERNEL(k_lshladd, OP_LSHLADD)
KERNEL(k_bfe, OP_BFE)
KERNEL(k_xad, OP_XAD)
KERNEL(k_fma, OP_FMA)
KERNEL(k_shl, OP_SHL)
KERNEL(k_shr, OP_SHR)
KERNEL(k_lshlor, OP_LSHLOR)
KERNEL(k_alignbyte, OP_ALIGNBYTE)
KERNEL(k_mov, OP_MOV)
KERNEL(k_bfi, OP_BFI)
KERNEL(k_or3, OP_OR3)
KERNEL(k_alignbit_same, OP_ALIGNBIT_SAME)
KERNEL(k_perm_same, OP_PERM_SAME)
KERNEL(k_xor_same, OP_XOR_SAME)
KERNEL(k_add_same, OP_ADD_SAME)

// 64-bit shifts and packed moves (rotate-by-64-bit-shift candidates).
__global__ __launch_bounds__(256) void k_lshr64(unsigned* out, int iters) {
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    for (int i = 0; i < iters; ++i) {
        asm volatile(REP8("v_lshrrev_b64 %0, 3, %0\n v_lshrrev_b64 %1, 3, %1\n"
                          "v_lshrrev_b64 %2, 3, %2\n v_lshrrev_b64 %3, 3, %3\n"
                          "v_lshrrev_b64 %0, 5, %0\n v_lshrrev_b64 %1, 5, %1\n"
                          "v_lshrrev_b64 %2, 5, %2\n v_lshrrev_b64 %3, 5, %3\n")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    }
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3);
}
__global__ __launch_bounds__(256) void k_pkmov(unsigned* out, int iters) {
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    for (int i = 0; i < iters; ++i) {
        asm volatile(REP8("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]\n v_pk_mov_b32 %1, %1, %1 op_sel:[1,0]\n"
                          "v_pk_mov_b32 %2, %2, %2 op_sel:[1,0]\n v_pk_mov_b32 %3, %3, %3 op_sel:[1,0]\n"
                          "v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]\n v_pk_mov_b32 %1, %1, %1 op_sel:[1,0]\n"
                          "v_pk_mov_b32 %2, %2, %2 op_sel:[1,0]\n v_pk_mov_b32 %3, %3, %3 op_sel:[1,0]\n")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    }
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3);
}

// 64-bit add forms used by SHA-512.
__global__ __launch_bounds__(256) void k_lshl_add_u64(unsigned* out, int iters) {
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned long long k = blockIdx.x | 1;
    for (int i = 0; i < iters; ++i) {
        asm volatile(REP8("v_lshl_add_u64 %0, %0, 0, %4\n v_lshl_add_u64 %1, %1, 0, %4\n"
                          "v_lshl_add_u64 %2, %2, 0, %4\n v_lshl_add_u64 %3, %3, 0, %4\n"
                          "v_lshl_add_u64 %0, %0, 0, %4\n v_lshl_add_u64 %1, %1, 0, %4\n"
                          "v_lshl_add_u64 %2, %2, 0, %4\n v_lshl_add_u64 %3, %3, 0, %4\n")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(k));
    }
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3);
}
__global__ __launch_bounds__(256) void k_addc_pair(unsigned* out, int iters) {
    unsigned l0 = threadIdx.x, h0 = 1, l1 = l0 + 3, h1 = 2;
    unsigned k = blockIdx.x | 1;
    for (int i = 0; i < iters; ++i) {
        asm volatile(REP8("v_add_co_u32 %0, vcc, %0, %4\n v_addc_co_u32 %1, vcc, %1, %4, vcc\n"
                          "v_add_co_u32 %2, vcc, %2, %4\n v_addc_co_u32 %3, vcc, %3, %4, vcc\n"
                          "v_add_co_u32 %0, vcc, %0, %4\n v_addc_co_u32 %1, vcc, %1, %4, vcc\n"
                          "v_add_co_u32 %2, vcc, %2, %4\n v_addc_co_u32 %3, vcc, %3, %4, vcc\n")
                     : "+v"(l0), "+v"(h0), "+v"(l1), "+v"(h1) : "v"(k) : "vcc");
    }
    out[blockIdx.x * 256 + threadIdx.x] = l0 ^ h0 ^ l1 ^ h1;
}

// Two DISTINCT live VGPR sources per instruction (as in r_a += r_b of a
// hash round), vs the single-live-source chains above.
#define PAIR8(OP) OP("%0", "%4") OP("%1", "%5") OP("%2", "%6") OP("%3", "%7") \
                  OP("%4", "%1") OP("%5", "%2") OP("%6", "%3") OP("%7", "%0")
#define P_ADD(d, s) "v_add_u32 " d ", " d ", " s "\n"
#define P_XOR(d, s) "v_xor_b32 " d ", " d ", " s "\n"
#define P_BITOP3(d, s) "v_bitop3_b32 " d ", " d ", " s ", %8 bitop3:0x96\n"
#define P_ADD3(d, s) "v_add3_u32 " d ", " d ", " s ", %8\n"
#define P_ALIGNBIT(d, s) "v_alignbit_b32 " d ", " d ", " s ", 7\n"
#define PAIRK(NAME, OP)                                                                   \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, int iters) {               \
        unsigned r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4,      \
                 r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;                                   \
        unsigned k0 = blockIdx.x | 1;                                                     \
        for (int i = 0; i < iters; ++i) {                                                 \
            asm volatile(REP8(PAIR8(OP))                                                  \
                         : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5),     \
                           "+v"(r6), "+v"(r7)                                              \
                         : "v"(k0));                                                      \
        }                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;       \
    }
PAIRK(kp_add, P_ADD)
PAIRK(kp_xor, P_XOR)
PAIRK(kp_bitop3, P_BITOP3)
PAIRK(kp_add3, P_ADD3)
PAIRK(kp_alignbit, P_ALIGNBIT)

// Mixes: full-rate add/xor with half-rate alignbit (the ChaCha / SHA mix).
#define MIX_G(OP) OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")
#define M_ADD(r) "v_add_u32 " r ", " r ", %8\n"
#define M_XOR(r) "v_xor_b32 " r ", " r ", %8\n"
#define M_ROT(r) "v_alignbit_b32 " r ", " r ", " r ", 7\n"
#define MIXK(NAME, BODY)                                                                   \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, int iters) {               \
        unsigned r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4,      \
                 r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;                                   \
        unsigned k0 = blockIdx.x | 1;                                                     \
        for (int i = 0; i < iters; ++i) {                                                 \
            asm volatile(BODY                                                             \
                         : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5),     \
                           "+v"(r6), "+v"(r7)                                              \
                         : "v"(k0));                                                      \
        }                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;       \
    }
// 2 full : 1 half, grouped by 8 chains (24 instructions per group) x 8 = 192
MIXK(km_grouped, REP8(MIX_G(M_ADD) MIX_G(M_XOR) MIX_G(M_ROT)))
// 1 full : 1 half
MIXK(km_1to1, REP8(MIX_G(M_XOR) MIX_G(M_ROT)))
// all full
MIXK(km_full, REP8(MIX_G(M_XOR) MIX_G(M_ADD)))

typedef void (*kfn)(unsigned*, int);

int main() {
    unsigned* out;
    hipMalloc(&out, 256 * 2048 * 8 * sizeof(unsigned));
    struct { const char* name; kfn f; int ninstr; } ks[] = {
        {"v_add_u32", k_add, 64}, {"v_add3_u32", k_add3, 64}, {"v_alignbit_b32", k_alignbit, 64},
        {"v_bitop3_b32", k_bitop3, 64}, {"v_xor_b32", k_xor, 64}, {"v_perm_b32", k_perm, 64},
        {"v_lshl_add_u32", k_lshladd, 64}, {"v_bfe_u32", k_bfe, 64}, {"v_xad_u32", k_xad, 64},
        {"v_fma_f32", k_fma, 64}, {"v_lshl_add_u64", k_lshl_add_u64, 64},
        {"v_add_co+addc (per instr)", k_addc_pair, 64},
        {"v_lshlrev_b32", k_shl, 64}, {"v_lshrrev_b32", k_shr, 64}, {"v_lshl_or_b32", k_lshlor, 64},
        {"v_alignbyte_b32", k_alignbyte, 64}, {"v_mov_b32", k_mov, 64}, {"v_bfi_b32", k_bfi, 64},
        {"v_or3_b32", k_or3, 64}, {"v_lshrrev_b64", k_lshr64, 64}, {"v_pk_mov_b32", k_pkmov, 64},
        {"v_alignbit_b32 x,x,x", k_alignbit_same, 64}, {"v_perm_b32 x,x,k", k_perm_same, 64},
        {"v_xor_b32 x,x", k_xor_same, 64}, {"v_add_u32 x,x", k_add_same, 64},
        {"2-live v_add_u32", kp_add, 64}, {"2-live v_xor_b32", kp_xor, 64},
        {"2-live v_bitop3_b32", kp_bitop3, 64}, {"2-live v_add3_u32", kp_add3, 64},
        {"2-live v_alignbit_b32", kp_alignbit, 64},
        {"mix add+xor+alignbit (2:1)", km_grouped, 192}, {"mix xor+alignbit (1:1)", km_1to1, 128},
        {"mix xor+add (full only)", km_full, 128}};
    int dev;
    hipGetDevice(&dev);
    int clk_khz;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves/SIMD
    const int iters = 4000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 10);
        hipDeviceSynchronize();
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // wave-instructions per SIMD: blocks*4 waves / (256 CU * 4 SIMD) * iters * ninstr
        double wi = (double)blocks * 4 / 1024.0 * iters * k.ninstr;
        double cyc_at_peak = ms * 1e-3 * clk_khz * 1e3;
        printf("%-28s %.3f ms  %.2f cycles/wave-instr/SIMD at %.0f MHz (lane-ops/s %.1f T)\n", k.name, ms,
               cyc_at_peak / wi, clk_khz / 1e3, wi * 1024 * 64 / (ms * 1e-3) / 1e12);
    }
    return 0;
}
