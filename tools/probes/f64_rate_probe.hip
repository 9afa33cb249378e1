// Probe 2: fp64 MFMA vs VALU issue rate with in-kernel clock (s_memtime / s_memrealtime @100MHz),
// and MFMA+VALU co-execution in one workgroup.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

__device__ inline void mfma_loop(int iters, double a, double b, d4* acc){
  for(int it=0; it<iters; it++){
#pragma unroll
    for(int i=0;i<4;i++) acc[i]=__builtin_amdgcn_mfma_f64_16x16x4f64(a,b,acc[i],0,0,0);
  }
}
__device__ inline double valu_loop(int iters, double s){
  double x0=s,x1=s+1,x2=s+2,x3=s+3,x4=s+4,x5=s+5,x6=s+6,x7=s+7;
  double m=1.0000001, c=1e-9;
  for(int it=0; it<iters; it++){
    x0=fma(x0,m,c);x1=fma(x1,m,c);x2=fma(x2,m,c);x3=fma(x3,m,c);
    x4=fma(x4,m,c);x5=fma(x5,m,c);x6=fma(x6,m,c);x7=fma(x7,m,c);
  }
  return x0+x1+x2+x3+x4+x5+x6+x7;
}
// mode 0: all waves MFMA; 1: all waves VALU; 2: waves with (wave&1)==0 MFMA, others VALU
__global__ void __launch_bounds__(256) rate_k(double* out, unsigned long long* clk, int mode, int iters_m, int iters_v){
  int w = threadIdx.x>>6;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  double res=0;
  bool do_m = (mode==0) || (mode==2 && (w&1)==0);
  if(do_m){ d4 acc[4]; for(int i=0;i<4;i++) acc[i]=(d4){0,0,0,0}; mfma_loop(iters_m, 1.0*threadIdx.x, 2.0, acc);
    for(int i=0;i<4;i++) res+=acc[i][0]+acc[i][1]+acc[i][2]+acc[i][3]; }
  else res = valu_loop(iters_v, 1.0*threadIdx.x);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x*blockDim.x+threadIdx.x]=res;
  if(threadIdx.x==0){ clk[blockIdx.x*2]=t1-t0; clk[blockIdx.x*2+1]=r1-r0; }
}
int main(){
  int ncu=256;
  double* dout; CK(hipMalloc(&dout,(size_t)ncu*8*256*8));
  unsigned long long* dclk; CK(hipMalloc(&dclk,(size_t)ncu*8*2*8));
  std::vector<unsigned long long> h(ncu*8*2);
  hipEvent_t e0,e1; CK(hipEventCreate(&e0));CK(hipEventCreate(&e1));
  const int IM=8000, IV=32000;
  for(int wpc : {1,2,4}){
    for(int mode : {0,1,2}){
      int grid=ncu*wpc;
      rate_k<<<grid,256>>>(dout,dclk,mode,100,400); CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0)); rate_k<<<grid,256>>>(dout,dclk,mode,IM,IV); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms,e0,e1));
      CK(hipMemcpy(h.data(),dclk,grid*2*8,hipMemcpyDeviceToHost));
      std::vector<double> ghz; for(int b=0;b<grid;b++) ghz.push_back((double)h[b*2]/(double)h[b*2+1]*0.1);
      std::sort(ghz.begin(),ghz.end()); double med=ghz[grid/2];
      double cyc = (double)h[0];
      double nm = (mode==0)? 4.0 : (mode==2? 2.0:0.0);  // mfma waves per WG
      double nv = (mode==1)? 4.0 : (mode==2? 2.0:0.0);
      double fm = (double)grid*nm*IM*4*2048.0, fv=(double)grid*nv*256.0/4*IV*8*2.0;
      printf("wg/cu=%d mode=%d: %.3f ms, clock(med)=%.2f GHz, MFMA %.1f TF + VALU %.1f TF = %.1f TF; cyc/MFMA(blk0)=%.1f cyc/8fma(blk0)=%.1f\n",
        wpc, mode, ms, med, fm/ms/1e9, fv/ms/1e9, (fm+fv)/ms/1e9, nm>0? cyc/(IM*4.0):0.0, nv>0&&nm==0? cyc/(double)IV:0.0);
    }
  }
  printf("PROBE2 DONE\n");
}
