// Microbenchmark: BN254 Fp Montgomery multiply throughput/latency on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
__constant__ uint32_t P[8] = {0xd87cfd47u,0x3c208c16u,0x6871ca8du,0x97816a91u,0x8181585du,0xb85045b6u,0xe131a029u,0x30644e72u};
#define NP0 0xe4866389u
__device__ __forceinline__ void mont_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t t[10];
  #pragma unroll
  for (int j=0;j<10;j++) t[j]=0;
  #pragma unroll
  for (int i=0;i<8;i++){
    uint64_t c=0;
    #pragma unroll
    for(int j=0;j<8;j++){ uint64_t s=(uint64_t)a[j]*b[i]+t[j]+c; t[j]=(uint32_t)s; c=s>>32; }
    uint64_t s=(uint64_t)t[8]+c; t[8]=(uint32_t)s; t[9]=(uint32_t)(s>>32);
    uint32_t m=t[0]*NP0;
    s=(uint64_t)m*P[0]+t[0]; c=s>>32;
    #pragma unroll
    for(int j=1;j<8;j++){ s=(uint64_t)m*P[j]+t[j]+c; t[j-1]=(uint32_t)s; c=s>>32; }
    s=(uint64_t)t[8]+c; t[7]=(uint32_t)s; t[8]=t[9]+(uint32_t)(s>>32);
  }
  // conditional subtract
  uint32_t d[8]; uint64_t br=0;
  #pragma unroll
  for(int j=0;j<8;j++){ uint64_t s=(uint64_t)t[j]-P[j]-br; d[j]=(uint32_t)s; br=(s>>63)&1; }
  bool ge = (t[8]!=0) || (br==0);
  #pragma unroll
  for(int j=0;j<8;j++) r[j]= ge? d[j]:t[j];
}
template<int ILP>
__global__ void k_fpmul(uint32_t* out, int iters) {
  uint32_t a[ILP][8], b[8];
  uint32_t tid = blockIdx.x*blockDim.x+threadIdx.x;
  #pragma unroll
  for(int k=0;k<ILP;k++)
  #pragma unroll
  for(int j=0;j<8;j++) a[k][j]= (tid*2654435761u + j*40503u + k*7u) & (j==7?0x0fffffffu:0xffffffffu);
  #pragma unroll
  for(int j=0;j<8;j++) b[j]= (tid*97u + j*13u+5u) & (j==7?0x0fffffffu:0xffffffffu);
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int k=0;k<ILP;k++) mont_mul(a[k],a[k],b);
  }
  uint32_t x=0;
  #pragma unroll
  for(int k=0;k<ILP;k++)
  #pragma unroll
  for(int j=0;j<8;j++) x^=a[k][j];
  out[tid]=x;
}
__global__ void k_mad(uint64_t* out, int iters){
  uint32_t tid = blockIdx.x*blockDim.x+threadIdx.x;
  uint64_t acc[8]; uint32_t x[8];
  #pragma unroll
  for(int j=0;j<8;j++){acc[j]=tid+j; x[j]=tid*3+j;}
  for(int it=0;it<iters;it++){
    #pragma unroll
    for(int j=0;j<8;j++) acc[j]=(uint64_t)x[j]*x[(j+1)&7]+acc[j];
    #pragma unroll
    for(int j=0;j<8;j++) x[j]^=(uint32_t)acc[j];
  }
  uint64_t s=0;
  #pragma unroll
  for(int j=0;j<8;j++) s+=acc[j];
  out[tid]=s;
}
int main(){
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop,0));
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  uint32_t* d; CK(hipMalloc(&d, 64<<20));
  hipEvent_t e0,e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int iters=2000;
  for (int blocks : {256, 1024, 4096, 16384}) {
    for (int bs : {64, 256}) {
      if ((long)blocks*bs*4 > (64<<20)) continue;
      hipLaunchKernelGGL(k_fpmul<1>, dim3(blocks), dim3(bs), 0, 0, d, 10);
      CK(hipDeviceSynchronize());
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_fpmul<1>, dim3(blocks), dim3(bs), 0, 0, d, iters);
      hipEventRecord(e1); CK(hipEventSynchronize(e1));
      float ms; hipEventElapsedTime(&ms,e0,e1);
      double muls=(double)blocks*bs*iters;
      printf("fpmul ILP1 blocks=%d bs=%d : %.3f ms  %.3f Gmul/s  per-wave-mul %.1f ns\n", blocks, bs, ms, muls/ms/1e6, ms*1e6/iters);
    }
  }
  for (int blocks : {1024, 4096, 16384}) {
    int bs=256;
    hipLaunchKernelGGL(k_fpmul<2>, dim3(blocks), dim3(bs), 0, 0, d, 10);
    CK(hipDeviceSynchronize());
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fpmul<2>, dim3(blocks), dim3(bs), 0, 0, d, iters);
    hipEventRecord(e1); CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms,e0,e1);
    double muls=(double)blocks*bs*iters*2;
    printf("fpmul ILP2 blocks=%d bs=%d : %.3f ms  %.3f Gmul/s\n", blocks, bs, ms, muls/ms/1e6);
  }
  // single wave latency
  {
    hipLaunchKernelGGL(k_fpmul<1>, dim3(1), dim3(64), 0, 0, d, 10);
    CK(hipDeviceSynchronize());
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fpmul<1>, dim3(1), dim3(64), 0, 0, d, iters);
    hipEventRecord(e1); CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms,e0,e1);
    printf("single wave: %.1f ns per dependent fpmul\n", ms*1e6/iters);
  }
  {
    uint64_t* d2; CK(hipMalloc(&d2, 64<<20));
    int blocks=16384, bs=256; int it2=4000;
    hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(bs), 0, 0, d2, 10);
    CK(hipDeviceSynchronize());
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(bs), 0, 0, d2, it2);
    hipEventRecord(e1); CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms,e0,e1);
    double mads=(double)blocks*bs*it2*8;
    printf("v_mad_u64_u32 peak probe: %.3f ms  %.1f Gmad/s (%.1f mad/clk/CU at 2.4GHz)\n", ms, mads/ms/1e6, mads/ms/1e6/2.4/256);
  }
  return 0;
}
