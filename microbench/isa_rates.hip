// Integer-VALU issue-rate microbenchmark for gfx950 (MI355X).
// Decides the field-arithmetic radix for the Ed25519 kernels (SURVEY.md §7 "hard parts":
// v_mad_u64_u32 throughput on gfx950 is unknown). Each lane runs NACC independent
// dependency chains of one instruction; the grid fills the chip at a chosen waves/SIMD.
// Output: wave-instructions/s and cycles per wave-instruction per SIMD at an assumed clock,
// normalised against v_add_u32 (full rate) measured in the same process.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int NACC = 8;
constexpr int ITERS = 65536;

#define BODY_MAD64(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc64[i]) : "v"(a[i]), "v"(b) : "vcc");
#define BODY_MULLO(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_MULHI(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_MUL24(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_MULHI24(i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_MAD24(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
#define BODY_ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_ADDC(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %1, vcc" : "+v"(a[i]), "+v"(c[i]) : "v"(b) : "vcc");
#define BODY_ALIGN(i) asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a[i]) : "v"(b));
#define BODY_FMA64(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d64[i]) : "v"(dx), "v"(dy));
#define BODY_DPP(i) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]));
#define BODY_CND(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc");
#define BODY_AND(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_OR(i) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_XOR(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_SHL(i) asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(a[i]));
#define BODY_SHR(i) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(a[i]));
#define BODY_SUB(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_ADDCO(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b) : "vcc");
#define BODY_LSHLADD64(i) asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(acc64[i]) : "v"(acc64[(i+1)&7]));
#define BODY_ADD3(i) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
#define BODY_LSHLOR(i) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[i]) : "v"(b));
#define BODY_ANDOR(i) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
#define BODY_MOV(i) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i+1)&7]));
#define BODY_CNDS(i) asm volatile("v_cndmask_b32 %0, %0, %1, s[20:21]" : "+v"(a[i]) : "v"(b) : "s20", "s21");
#define BODY_BFI(i) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
#define BODY_PERM(i) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
#define BODY_ADDF32(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_PKADD16(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BODY_ADDLIT(i) asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a[i]));
#define BODY_LSHR64(i) asm volatile("v_lshrrev_b64 %0, 26, %0" : "+v"(acc64[i]));
#define BODY_BFE(i) asm volatile("v_bfe_u32 %0, %0, 3, 26" : "+v"(a[i]) : );

#define REP8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)

#define KERNEL(NAME, M)                                                          \
__global__ void NAME(uint32_t* out, uint32_t seed) {                              \
  uint32_t a[NACC], c[NACC]; uint64_t acc64[NACC]; double d64[NACC];             \
  uint32_t b = seed ^ threadIdx.x; double dx = 1.0000001 + threadIdx.x, dy = 0.9999; \
  for (int i = 0; i < NACC; ++i) { a[i] = seed * (i + 3) + threadIdx.x; c[i] = i;  \
    acc64[i] = a[i]; d64[i] = a[i]; }                                             \
  for (int it = 0; it < ITERS; ++it) { REP8(M) }                                  \
  uint32_t r = 0; for (int i = 0; i < NACC; ++i)                                  \
    r ^= a[i] ^ c[i] ^ (uint32_t)acc64[i] ^ (uint32_t)(acc64[i] >> 32) ^ (uint32_t)d64[i]; \
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                 \
}

KERNEL(k_mad64, BODY_MAD64)
KERNEL(k_mullo, BODY_MULLO)
KERNEL(k_mulhi, BODY_MULHI)
KERNEL(k_mul24, BODY_MUL24)
KERNEL(k_mulhi24, BODY_MULHI24)
KERNEL(k_mad24, BODY_MAD24)
KERNEL(k_add, BODY_ADD)
KERNEL(k_addc, BODY_ADDC)
KERNEL(k_align, BODY_ALIGN)
KERNEL(k_fma64, BODY_FMA64)
KERNEL(k_dpp, BODY_DPP)
KERNEL(k_cnd, BODY_CND)
KERNEL(k_lshr64, BODY_LSHR64)
KERNEL(k_and, BODY_AND)
KERNEL(k_or, BODY_OR)
KERNEL(k_xor, BODY_XOR)
KERNEL(k_shl, BODY_SHL)
KERNEL(k_shr, BODY_SHR)
KERNEL(k_sub, BODY_SUB)
KERNEL(k_addco, BODY_ADDCO)
KERNEL(k_lshladd64, BODY_LSHLADD64)
KERNEL(k_add3, BODY_ADD3)
KERNEL(k_lshlor, BODY_LSHLOR)
KERNEL(k_andor, BODY_ANDOR)
KERNEL(k_mov, BODY_MOV)
KERNEL(k_cnds, BODY_CNDS)
KERNEL(k_bfi, BODY_BFI)
KERNEL(k_perm, BODY_PERM)
KERNEL(k_addf32, BODY_ADDF32)
KERNEL(k_pkadd16, BODY_PKADD16)
KERNEL(k_addlit, BODY_ADDLIT)
KERNEL(k_bfe, BODY_BFE)

typedef void (*kfn)(uint32_t*, uint32_t);
struct Entry { const char* name; kfn f; int instrs_per_body; };

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"gcn\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.name, prop.gcnArchName, cus, prop.clockRate);
  Entry es[] = {{"v_add_u32", k_add, 1}, {"v_mad_u64_u32", k_mad64, 1}, {"v_mul_lo_u32", k_mullo, 1},
                {"v_mul_hi_u32", k_mulhi, 1}, {"v_mul_u32_u24", k_mul24, 1}, {"v_mul_hi_u32_u24", k_mulhi24, 1},
                {"v_mad_u32_u24", k_mad24, 1}, {"v_add_co+v_addc_co", k_addc, 2}, {"v_alignbit_b32", k_align, 1},
                {"v_fma_f64", k_fma64, 1}, {"v_mov_b32_dpp", k_dpp, 1}, {"v_cndmask_b32", k_cnd, 1},
                {"v_lshrrev_b64", k_lshr64, 1}, {"v_bfe_u32", k_bfe, 1},
                {"v_and_b32", k_and, 1}, {"v_or_b32", k_or, 1}, {"v_xor_b32", k_xor, 1}, {"v_lshlrev_b32", k_shl, 1},
                {"v_lshrrev_b32", k_shr, 1}, {"v_sub_u32", k_sub, 1}, {"v_add_co_u32", k_addco, 1},
                {"v_lshl_add_u64", k_lshladd64, 1}, {"v_add3_u32", k_add3, 1}, {"v_lshl_or_b32", k_lshlor, 1},
                {"v_and_or_b32", k_andor, 1}, {"v_mov_b32", k_mov, 1}, {"v_cndmask_b32(sgpr)", k_cnds, 1},
                {"v_bfi_b32", k_bfi, 1}, {"v_perm_b32", k_perm, 1}, {"v_add_f32", k_addf32, 1},
                {"v_pk_add_u16", k_pkadd16, 1}, {"v_add_u32(literal)", k_addlit, 1}};
  uint32_t* out; size_t maxthreads = (size_t)cus * 4 * 8 * 64;
  CHECK(hipMalloc(&out, maxthreads * 4));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  double add_rate[9] = {0};
  (void)0;
  for (int wps : {2, 4, 8}) {
    for (auto& e : es) {
      int threads = 256;  // 4 waves per block -> one per SIMD
      int blocks = cus * wps;
      hipLaunchKernelGGL(e.f, dim3(blocks), dim3(threads), 0, 0, out, 12345u);  // warm
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      const int reps = 3;
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(e.f, dim3(blocks), dim3(threads), 0, 0, out, 777u + r);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      double waveinstr = (double)reps * blocks * 4 * ITERS * NACC * e.instrs_per_body;
      double rate = waveinstr / (ms * 1e-3);  // wave-instructions per second, whole chip
      if (!strcmp(e.name, "v_add_u32")) add_rate[wps] = rate;
      double cyc_at_24 = (double)cus * 4 * 2.4e9 / rate;  // cycles per wave-instr per SIMD at 2.4 GHz
      printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"wave_instr_per_s\": %.4g, "
             "\"cyc_per_wave_instr_at_2.4GHz\": %.2f, \"rel_to_add\": %.3f}\n",
             e.name, wps, ms, rate, cyc_at_24, add_rate[wps] / rate);
    }
  }
  return 0;
}
