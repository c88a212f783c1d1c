// Probe: does an out-of-range lane of buffer_load_dwordx4 ... lds write ZEROS into its LDS
// slot on gfx950 (raw buffer, offset >= num_records), or leave the slot untouched?
// Build: hipcc --offload-arch=gfx950 -O3 buffer_lds_oob_probe.hip -o buffer_lds_oob_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((address_space(3))) void lds_void;
__global__ void probe(const short* p, unsigned nbytes, short* out) {
  __shared__ short s[64 * 8];
  for (int j = 0; j < 8; ++j) s[threadIdx.x * 8 + j] = 0x7777;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)nbytes, 0x00020000);
  unsigned off = threadIdx.x * 16;
  if (threadIdx.x & 1) off = nbytes;  // out of range
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)s, 16, off, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int j = 0; j < 8; ++j) out[threadIdx.x * 8 + j] = s[threadIdx.x * 8 + j];
}
int main() {
  short h[512], *d, *o;
  for (int i = 0; i < 512; ++i) h[i] = (short)(i + 1);
  hipMalloc(&d, 1024);
  hipMalloc(&o, 1024);
  hipMemcpy(d, h, 1024, hipMemcpyHostToDevice);
  probe<<<1, 64>>>(d, 1024, o);
  short r[512];
  hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
  int zero = 0, stale = 0, data = 0, bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 8; ++j) {
      const short v = r[l * 8 + j];
      if (l & 1) {
        if (v == 0) ++zero; else if (v == 0x7777) ++stale; else ++bad;
      } else {
        if (v == h[l * 8 + j]) ++data; else ++bad;
      }
    }
  printf("in-range lanes correct: %d/256; out-of-range slots: zero %d stale %d other %d; bad %d\n", data, zero, stale,
         256 - zero - stale, bad);
  return 0;
}
