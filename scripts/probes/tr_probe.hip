// Probe: empirical lane mapping of ds_read_b64_tr_b16 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void probe(short* out, int mode) {
  __shared__ short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = (short)i;  // value = row*64 + col
  __syncthreads();
  int l = threadIdx.x, i = l & 15, g = l >> 4, q = i >> 2, p = i & 3;
  int row = q, col = 4 * p;
  if (mode == 1) { row = 4 * g + q; col = 4 * p; }
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + row * 64 + col));
  for (int k = 0; k < 4; ++k) out[l * 4 + k] = r[k];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  short h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mode %d (value=row*64+col)\n", mode);
    for (int l = 0; l < 64; ++l) {
      printf("lane %2d:", l);
      for (int k = 0; k < 4; ++k) printf(" (%d,%d)", h[l * 4 + k] / 64, h[l * 4 + k] % 64);
      printf("\n");
    }
  }
  return 0;
}
