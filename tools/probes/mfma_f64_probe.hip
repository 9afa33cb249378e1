// Probe: fp64 MFMA (v_mfma_f64_16x16x4_f64) operand/result lane maps and throughput on gfx950,
// plus the fp64 VALU FMA rate. Results feed DESIGN.md (peak used for roofline.frac).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

// A is 16x4 (row-major), B is 4x16 (row-major). lane l loads a per hypothesis A[l&15][l>>4], B[l>>4][l&15]
__global__ void layout_k(const double* A, const double* B, double* C){
  int l = threadIdx.x;
  double a = A[(l&15)*4 + (l>>4)];
  double b = B[(l>>4)*16 + (l&15)];
  d4 acc = {0,0,0,0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0,0,0);
  for(int r=0;r<4;r++) C[l*4+r]=acc[r];
}

template<int NACC>
__global__ void __launch_bounds__(256) mfma_rate(double* out, int iters, double s){
  d4 acc[NACC];
  for(int i=0;i<NACC;i++) acc[i]=(d4){0,0,0,0};
  double a = s*threadIdx.x, b = s+threadIdx.x;
  for(int it=0; it<iters; it++){
#pragma unroll
    for(int i=0;i<NACC;i++) acc[i]=__builtin_amdgcn_mfma_f64_16x16x4f64(a,b,acc[i],0,0,0);
  }
  double t=0; for(int i=0;i<NACC;i++) t+=acc[i][0]+acc[i][1]+acc[i][2]+acc[i][3];
  out[blockIdx.x*blockDim.x+threadIdx.x]=t;
}

__global__ void __launch_bounds__(256) fma_rate(double* out, int iters, double s){
  double x0=s,x1=s+1,x2=s+2,x3=s+3,x4=s+4,x5=s+5,x6=s+6,x7=s+7;
  double m=1.0000001, c=1e-9;
  for(int it=0; it<iters; it++){
    x0=fma(x0,m,c);x1=fma(x1,m,c);x2=fma(x2,m,c);x3=fma(x3,m,c);
    x4=fma(x4,m,c);x5=fma(x5,m,c);x6=fma(x6,m,c);x7=fma(x7,m,c);
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=x0+x1+x2+x3+x4+x5+x6+x7;
}
__global__ void empty_k(double* out){ if(threadIdx.x==1234567) out[0]=1; }

int main(){
  // ---- layout
  std::vector<double> A(64), B(64), C(256);
  for(int i=0;i<16;i++) for(int k=0;k<4;k++) A[i*4+k] = (i+1) + 100.0*(k+1)*(k==0?0:1) ; // distinct-ish
  // use exact-integer random matrices
  srand(1);
  for(auto& v:A) v = (double)(rand()%17 - 8);
  for(auto& v:B) v = (double)(rand()%13 - 6);
  double *dA,*dB,*dC; CK(hipMalloc(&dA,64*8));CK(hipMalloc(&dB,64*8));CK(hipMalloc(&dC,256*8));
  CK(hipMemcpy(dA,A.data(),64*8,hipMemcpyHostToDevice));CK(hipMemcpy(dB,B.data(),64*8,hipMemcpyHostToDevice));
  layout_k<<<1,64>>>(dA,dB,dC); CK(hipDeviceSynchronize());
  CK(hipMemcpy(C.data(),dC,256*8,hipMemcpyDeviceToHost));
  double ref[16][16]; for(int i=0;i<16;i++)for(int j=0;j<16;j++){double s=0;for(int k=0;k<4;k++) s+=A[i*4+k]*B[k*16+j]; ref[i][j]=s;}
  int okH1=1, okH2=1;
  for(int l=0;l<64;l++) for(int r=0;r<4;r++){
    int col=l&15;
    int rowH1=(l>>4)+4*r;      // guide: row=(lane>>4)+4*reg
    int rowH2=4*(l>>4)+r;      // f32-style: row=4*(lane>>4)+reg
    if(C[l*4+r]!=ref[rowH1][col]) okH1=0;
    if(C[l*4+r]!=ref[rowH2][col]) okH2=0;
  }
  printf("LAYOUT row=(lane>>4)+4*reg: %s ; row=4*(lane>>4)+reg: %s\n", okH1?"MATCH":"no", okH2?"MATCH":"no");

  // ---- throughput
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p,0));
  int ncu=p.multiProcessorCount; printf("CUs=%d clock=%d kHz name=%s arch=%s\n",ncu,p.clockRate,p.name,p.gcnArchName);
  double* dout; CK(hipMalloc(&dout, (size_t)ncu*8*256*8));
  hipEvent_t e0,e1; CK(hipEventCreate(&e0));CK(hipEventCreate(&e1));
  int iters=4000;
  for(int wg_per_cu : {1,2,4}){
    int grid=ncu*wg_per_cu;
    mfma_rate<4><<<grid,256>>>(dout,10,1.0); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); mfma_rate<4><<<grid,256>>>(dout,iters,1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms,e0,e1));
    double flops=(double)grid*4/*waves*/*iters*4/*acc*/*2048.0;
    printf("MFMA f64 16x16x4 NACC=4 wg/cu=%d: %.2f TFLOP/s (%.3f ms)\n",wg_per_cu, flops/ms/1e9, ms);
    mfma_rate<8><<<grid,256>>>(dout,10,1.0); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); mfma_rate<8><<<grid,256>>>(dout,iters,1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms,e0,e1));
    flops=(double)grid*4*iters*8*2048.0;
    printf("MFMA f64 16x16x4 NACC=8 wg/cu=%d: %.2f TFLOP/s (%.3f ms)\n",wg_per_cu, flops/ms/1e9, ms);
    CK(hipEventRecord(e0)); fma_rate<<<grid,256>>>(dout,iters*4,1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms,e0,e1));
    flops=(double)grid*256*iters*4*8*2.0;
    printf("VALU f64 fma wg/cu=%d: %.2f TFLOP/s (%.3f ms)\n",wg_per_cu, flops/ms/1e9, ms);
  }
  // ---- launch gap
  for(int i=0;i<10;i++) empty_k<<<256,256>>>(dout); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); for(int i=0;i<1000;i++) empty_k<<<256,256>>>(dout); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms,e0,e1)); printf("empty kernel back-to-back: %.2f us/launch\n", ms);
  // graph
  hipStream_t s; CK(hipStreamCreate(&s)); hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s,hipStreamCaptureModeGlobal)); for(int i=0;i<1000;i++) empty_k<<<256,256,0,s>>>(dout); CK(hipStreamEndCapture(s,&g));
  CK(hipGraphInstantiate(&ge,g,nullptr,nullptr,0)); CK(hipGraphLaunch(ge,s)); CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0,s)); CK(hipGraphLaunch(ge,s)); CK(hipEventRecord(e1,s)); CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms,e0,e1)); printf("empty kernel in graph: %.2f us/launch\n", ms);
  printf("PROBE DONE\n");
  return 0;
}
