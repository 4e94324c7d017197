#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
__global__ void add1(float* x, int n){ int i=blockIdx.x*blockDim.x+threadIdx.x; if(i<n) x[i]+=1.0f; }
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void mfma_test(const short* A, const short* B, float* C){
  // 16x16x32: A[16][32] row-major, B[32][16] (k-major), C[16][16]
  int l=threadIdx.x;
  bf16x8 a,b;
  for(int j=0;j<8;j++){ a[j]=A[(l&15)*32 + 8*(l>>4)+j]; b[j]=B[(8*(l>>4)+j)*16 + (l&15)]; }
  f32x4 c={0,0,0,0};
  c=__builtin_amdgcn_mfma_f32_16x16x32_bf16(a,b,c,0,0,0);
  for(int j=0;j<4;j++) C[((l>>4)*4+j)*16 + (l&15)] = c[j];
}
extern "C" int launch_add1(void* x, int n, void* stream){ hipLaunchKernelGGL(add1, dim3((n+255)/256), dim3(256), 0, (hipStream_t)stream, (float*)x, n); return (int)hipGetLastError(); }
extern "C" int launch_mfma(void* A, void* B, void* C, void* stream){ hipLaunchKernelGGL(mfma_test, dim3(1), dim3(64), 0, (hipStream_t)stream, (const short*)A,(const short*)B,(float*)C); return (int)hipGetLastError(); }
