// Probe: issue rate (independent) and dependent-chain latency of the VALU instructions the search
// kernel is made of, on gfx950.  Each wave runs ITER x 8 instructions of one kind on 8 independent
// registers (rate) or one chain (latency); printed as SIMD cycles per wave-instruction, derived
// from wall time at the measured clock: cycles = time * clock * SIMDs / (waves * instructions).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITER 512
#define BODY8(ins) ins(a0) ins(a1) ins(a2) ins(a3) ins(a4) ins(a5) ins(a6) ins(a7)
#define K(name, ins)                                                                         \
  __global__ void name(uint32_t* out, uint32_t s) {                                          \
    const uint64_t msk = 0x5555555555555555ull + s;                                          \
    uint32_t a0 = s + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, \
             a6 = a0 * 13, a7 = a0 ^ 15, b = s * 17 + threadIdx.x, c = s * 19;                \
    for (int i = 0; i < ITER; i++) { BODY8(ins) }                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;       \
  }
#define I_DOT4C(r) asm volatile("v_dot4c_i32_i8 %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_DOT4(r) asm volatile("v_dot4_i32_i8 %0, %1, %2, %0" : "+v"(r) : "v"(b), "v"(c));
#define I_DOT2C(r) asm volatile("v_dot2c_i32_i16 %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_DOT2(r) asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(r) : "v"(b), "v"(c));
#define I_PKSUB(r) asm volatile("v_pk_sub_i16 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_PKADD(r) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_PKMAX(r) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_PKMAD(r) asm volatile("v_pk_mad_u16 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_PERM(r) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_ALIGN(r) asm volatile("v_alignbyte_b32 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_ADD(r) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_MED3(r) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_SAD(r) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(r) : "v"(b), "v"(c));
#define I_DPP(r) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r));
#define I_MOV(r) asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(b));
#define I_CND(r) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r) : "v"(b));
#define I_CND64(r) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r) : "v"(b), "s"(msk));
#define I_CNDV(r) asm volatile("v_cmp_lt_u32 vcc, %1, %2\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r) : "v"(b), "v"(c) : "vcc");
#define I_AND(r) asm volatile("v_and_b32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_OR(r) asm volatile("v_or_b32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_LSHR(r) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(r));
#define I_LSHLV(r) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(r) : "v"(c));
#define I_MIN(r) asm volatile("v_min_i32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_ADDF(r) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_PKFMA(r) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(r64) : "v"(b64), "v"(c64));
#define I_XOR(r) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_LSHL(r) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(r));
#define I_ASHR(r) asm volatile("v_ashrrev_i32 %0, 3, %0" : "+v"(r));
#define I_MAX(r) asm volatile("v_max_i32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_ADD3(r) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_LSHLADD(r) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(r) : "v"(b));
#define I_MAD24(r) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_MULLO(r) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_BFE(r) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(r));
#define I_PKMUL(r) asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_UDOT2(r) asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(r) : "v"(b), "v"(c));
#define I_FMA(r) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_MUL24(r) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_SDWA(r) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(r) : "v"(b));
#define I_ADDDPP(r) asm volatile("v_add_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r));
#define I_SUBREV(r) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(r) : "v"(b));
#define I_PKADDI(r) asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_CVTPK(r) asm volatile("v_cvt_pk_i16_i32 %0, %0, %1" : "+v"(r) : "v"(b));
#define I_PACK(r) asm volatile("v_pack_b32_f16 %0, %0, %1" : "+v"(r) : "v"(b));
K(k_dot4c, I_DOT4C) K(k_dot4, I_DOT4) K(k_dot2c, I_DOT2C) K(k_dot2, I_DOT2) K(k_pksub, I_PKSUB)
K(k_pkadd, I_PKADD) K(k_pkmax, I_PKMAX) K(k_pkmad, I_PKMAD) K(k_perm, I_PERM) K(k_align, I_ALIGN)
K(k_add, I_ADD) K(k_med3, I_MED3) K(k_sad, I_SAD) K(k_dpp, I_DPP)
K(k_mov, I_MOV) K(k_cnd, I_CND) K(k_xor, I_XOR) K(k_lshl, I_LSHL) K(k_ashr, I_ASHR) K(k_max, I_MAX) K(k_add3, I_ADD3)
K(k_lshladd, I_LSHLADD) K(k_mad24, I_MAD24) K(k_mullo, I_MULLO) K(k_bfe, I_BFE) K(k_pkmul, I_PKMUL) K(k_udot2, I_UDOT2)
K(k_fma, I_FMA) K(k_mul24, I_MUL24) K(k_sdwa, I_SDWA) K(k_adddpp, I_ADDDPP) K(k_subrev, I_SUBREV) K(k_pkaddi, I_PKADDI)
K(k_cvtpk, I_CVTPK) K(k_pack, I_PACK) K(k_cnd64, I_CND64) K(k_cndv, I_CNDV) K(k_and, I_AND) K(k_or, I_OR)
K(k_lshr, I_LSHR) K(k_lshlv, I_LSHLV) K(k_min, I_MIN) K(k_addf, I_ADDF)
// dependent chain: one register
#define KD(name, ins)                                                                        \
  __global__ void name(uint32_t* out, uint32_t s) {                                          \
    uint32_t a0 = s + threadIdx.x, b = s * 17 + threadIdx.x, c = s * 19;                     \
    for (int i = 0; i < ITER; i++) { ins(a0) ins(a0) ins(a0) ins(a0) ins(a0) ins(a0) ins(a0) ins(a0) } \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0;                                         \
  }
KD(d_dot4c, I_DOT4C) KD(d_dot2c, I_DOT2C) KD(d_pksub, I_PKSUB) KD(d_perm, I_PERM) KD(d_add, I_ADD) KD(d_align, I_ALIGN)

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  int cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   // kHz
  uint32_t* out;
  (void)hipMalloc(&out, sizeof(uint32_t) * 4096 * 1024);
  struct { const char* n; kfn f; } ks[] = {
    {"dot4c", k_dot4c}, {"dot4(vop3p)", k_dot4}, {"dot2c", k_dot2c}, {"dot2(vop3p)", k_dot2}, {"pk_sub_i16", k_pksub},
    {"pk_add_u16", k_pkadd}, {"pk_max_i16", k_pkmax}, {"pk_mad_u16", k_pkmad}, {"perm", k_perm}, {"alignbyte", k_align},
    {"add_u32", k_add}, {"med3_i32", k_med3}, {"sad_u8", k_sad}, {"mov_dpp", k_dpp},
    {"mov_b32", k_mov}, {"cndmask", k_cnd}, {"xor", k_xor}, {"lshlrev", k_lshl}, {"ashrrev", k_ashr}, {"max_i32", k_max},
    {"add3_u32", k_add3}, {"lshl_add", k_lshladd}, {"mad_u32_u24", k_mad24}, {"mul_lo_u32", k_mullo}, {"bfe_u32", k_bfe},
    {"pk_mul_lo_u16", k_pkmul}, {"dot2_u32_u16", k_udot2}, {"fma_f32", k_fma}, {"mul_i32_i24", k_mul24},
    {"add_u32_sdwa", k_sdwa}, {"add_u32_dpp", k_adddpp}, {"sub_u32", k_subrev}, {"pk_add_i16", k_pkaddi},
    {"cvt_pk_i16_i32", k_cvtpk}, {"pack_b32_f16", k_pack}, {"cndmask_e64(s)", k_cnd64}, {"cmp+cndmask(vcc)", k_cndv},
    {"and_b32", k_and}, {"or_b32", k_or}, {"lshrrev", k_lshr}, {"lshlrev(v)", k_lshlv}, {"min_i32", k_min}, {"add_f32", k_addf},
    {"DEP dot4c", d_dot4c}, {"DEP dot2c", d_dot2c}, {"DEP pk_sub", d_pksub}, {"DEP perm", d_perm}, {"DEP add", d_add},
    {"DEP alignbyte", d_align}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int wpsimd : {2, 8}) {
    const int threads = 256, blocks = cus * wpsimd;   // 4 waves per block = one per SIMD
    printf("waves/SIMD %d (clock attr %d MHz)\n", wpsimd, clk / 1000);
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, 0);
      for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)r);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
      const double inst = 5.0 * blocks * 4 * ITER * 8;   // wave-instructions
      const double simd_cycles = ms * 1e-3 * 2.1e9 * cus * 4;  // at an assumed 2.1 GHz
      printf("  %-14s %7.3f ms  %5.2f SIMD-cycles per wave-instruction (2.1 GHz)\n", k.n, ms, simd_cycles / inst);
    }
  }
  return 0;
}
