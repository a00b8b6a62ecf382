// Probe: gfx950 fp8 (e4m3) widening instructions vs torch's float8_e4m3fn values.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned* in, float* out_f32, float* out_bf) {
  unsigned v = in[threadIdx.x];
  f2 a = __builtin_amdgcn_cvt_pk_f32_fp8(v, false);
  f2 b = __builtin_amdgcn_cvt_pk_f32_fp8(v, true);
  bf2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v, 1.0f, false);
  bf2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v, 1.0f, true);
  float* o = out_f32 + threadIdx.x * 4;
  o[0] = a[0]; o[1] = a[1]; o[2] = b[0]; o[3] = b[1];
  float* p = out_bf + threadIdx.x * 4;
  p[0] = (float)c[0]; p[1] = (float)c[1]; p[2] = (float)d[0]; p[3] = (float)d[1];
}
int main() {
  // bytes: 0x38 = 1.0, 0x40 = 2.0, 0xB8 = -1.0, 0x7E = 448, 0x01 = 2^-9, 0x3C = 1.5, 0x44 = 3.0, 0x30 = 0.5
  unsigned h[2] = {0xB8403038u, 0x3C017E44u};
  unsigned* d_in; float *d_a, *d_b;
  hipMalloc(&d_in, 8); hipMalloc(&d_a, 32); hipMalloc(&d_b, 32);
  hipMemcpy(d_in, h, 8, hipMemcpyHostToDevice);
  k<<<1, 2>>>(d_in, d_a, d_b);
  float a[8], b[8];
  hipMemcpy(a, d_a, 32, hipMemcpyDeviceToHost); hipMemcpy(b, d_b, 32, hipMemcpyDeviceToHost);
  printf("bytes (LE): 38 30 40 B8 | 44 7E 01 3C  expect 0.5? no: 0x38=1.0 0x30=0.5 0x40=2 0xB8=-1 | 0x44=3 0x7E=448 0x01=0.00195 0x3C=1.5\n");
  printf("cvt_pk_f32_fp8        :"); for (int i = 0; i < 8; ++i) printf(" %g", a[i]); printf("\n");
  printf("cvt_scalef32_pk_bf16  :"); for (int i = 0; i < 8; ++i) printf(" %g", b[i]); printf("\n");
  return 0;
}
