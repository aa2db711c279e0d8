// stepbench.hip -- ceiling of the headline step's exact HBM pattern (calibration, not product).
//
// The db4 J=6 4096 x 4096 fp64 step (bench.py): the forward reads x (1 plane) and writes
// d_1..d_6, a_6 (7 planes) with the sc1 store policy (vw_device.h VW_FWD_STORE_AUX = 16); the inverse
// reads those 7 planes non-temporally and writes y (1 plane) non-temporally.  Here the same bytes move
// with no arithmetic: one 512-thread workgroup per 4096-sample row, 4 x 16-byte vectors per thread,
// over R rotated buffer sets (R x 128 MiB of inputs >= 512 MiB, as bench.py --rotate), K steps timed
// with HIP events, on 1 stream or with the rows split over S streams (bench.py's contexts schedule).
//   ./stepbench [S]   -> JSON lines: pattern, ms per step, Msamples/s, GB/s (2.147 GB per step)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

// AUX: buffer-store cache policy (16 = sc1 as the forward's coefficient rows, 2 = nt, 0 = write-back)
template <int AUX>
__global__ void __launch_bounds__(512) fanout(const double* __restrict__ x, double* __restrict__ out, int N,
                                              long long plane, int J, long long row0) {
  const long long b = row0 + blockIdx.x;
  extern __shared__ double lds_hold[];  // the LDS footprint of the product kernels (argv[2]), never used
  if (N < 0) lds_hold[threadIdx.x] = 0;
  const int nv = N / 2;
  d2 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(x + b * N) + threadIdx.x + k * 512);
  for (int j = 0; j < J; ++j) {
    const double* row = out + j * plane + b * N;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int w = threadIdx.x + k * 512;
      if (w < nv) {
        const d2 o = v[k] * (double)(j + 1);
        if constexpr (AUX < 0) __builtin_nontemporal_store(o, reinterpret_cast<d2*>(const_cast<double*>(row)) + w);
        else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4, o), rsrc(row), w * 16, 0, AUX);
      }
    }
  }
}

__global__ void __launch_bounds__(512) fanin(const double* __restrict__ in, double* __restrict__ y, int N,
                                             long long plane, int J, long long row0) {
  const long long b = row0 + blockIdx.x;
  extern __shared__ double lds_hold[];
  if (N < 0) lds_hold[threadIdx.x] = 0;
  d2 acc[4] = {};
  for (int j = 0; j < J; ++j) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      acc[k] += __builtin_nontemporal_load(reinterpret_cast<const d2*>(in + j * plane + b * N) + threadIdx.x + k * 512);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(acc[k], reinterpret_cast<d2*>(y + b * N) + threadIdx.x + k * 512);
}

int main(int argc, char** argv) {
  const int B = 4096, N = 4096, J = 7, R = 4, K = 20, WARM = 40;
  const long long plane = (long long)B * N;
  // ./stepbench S LDS_FWD LDS_INV STAGGER: coefficient planes STAGGER doubles apart beyond B*N (0: contiguous)
  const long long pstr = plane + (argc > 4 ? atoll(argv[4]) : 0);
  struct Set { double *x, *c, *y; };
  std::vector<Set> sets(R);
  for (auto& s : sets) {
    CHK(hipMalloc(&s.x, plane * 8));
    CHK(hipMalloc(&s.c, pstr * 8 * J));
    CHK(hipMalloc(&s.y, plane * 8));
    CHK(hipMemset(s.x, 0, plane * 8));
    CHK(hipMemset(s.c, 0, pstr * 8 * J));
  }
  const double step_bytes = plane * 8.0 * 16;  // 1 + 7 planes forward, 7 + 1 inverse
  int smax = argc > 1 ? atoi(argv[1]) : 4;
  // ./stepbench S LDS_FWD LDS_INV: graph mode only, each workgroup holding that much LDS (bytes) -- the
  // product kernels' footprint (persistent forward: two level buffers; inverse: one), so that the streams'
  // passes can share a CU only as far as the product's can
  const int lds_f = argc > 2 ? atoi(argv[2]) : 0, lds_i = argc > 3 ? atoi(argv[3]) : 0;
  CHK(hipFuncSetAttribute((const void*)fanout<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHK(hipFuncSetAttribute((const void*)fanin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  std::vector<hipStream_t> st(8);
  for (auto& s : st) CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  std::vector<hipEvent_t> done(8);
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (auto& e : done) CHK(hipEventCreate(&e));

  auto run = [&](const char* name, int S, auto fwd) {
    // S parts of B / S rows, part p on stream p; K steps, step i on set i mod R
    auto issue = [&](int steps) {
      for (int i = 0; i < steps; ++i) {
        const Set& s = sets[i % R];
        for (int p = 0; p < S; ++p) {
          const long long rows = B / S, r0 = p * rows;
          fwd(s, rows, r0, st[p]);
          hipLaunchKernelGGL(fanin, dim3((unsigned)rows), dim3(512), 0, st[p], s.c, s.y, N, pstr, J, r0);
        }
      }
    };
    issue(WARM);
    CHK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(e0, st[0]));
      for (int p = 1; p < S; ++p) CHK(hipStreamWaitEvent(st[p], e0, 0));
      issue(K);
      for (int p = 1; p < S; ++p) {
        CHK(hipEventRecord(done[p], st[p]));
        CHK(hipStreamWaitEvent(st[0], done[p], 0));
      }
      CHK(hipEventRecord(e1, st[0]));
      CHK(hipEventSynchronize(e1));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      const double per = ms / K;
      printf("{\"pattern\": \"%s\", \"streams\": %d, \"rep\": %d, \"ms_per_step\": %.4f, \"Msamples_per_s\": %.1f, "
             "\"GBps\": %.1f}\n", name, S, rep, per, plane / (per * 1e-3) / 1e6, step_bytes / (per * 1e-3) / 1e9);
      fflush(stdout);
    }
  };
  // the same steps recorded per stream into one HIP graph each (bench.py --launch graph-k), replayed once
  auto run_graph = [&](int S) {
    std::vector<hipGraphExec_t> ex(S);
    for (int p = 0; p < S; ++p) {
      CHK(hipStreamBeginCapture(st[p], hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < K; ++i) {
        const Set& s = sets[i % R];
        const long long rows = B / S, r0 = p * rows;
        hipLaunchKernelGGL(fanout<16>, dim3((unsigned)rows), dim3(512), lds_f, st[p], s.x, s.c, N, pstr, J, r0);
        hipLaunchKernelGGL(fanin, dim3((unsigned)rows), dim3(512), lds_i, st[p], s.c, s.y, N, pstr, J, r0);
      }
      hipGraph_t g;
      CHK(hipStreamEndCapture(st[p], &g));
      CHK(hipGraphInstantiate(&ex[p], g, nullptr, nullptr, 0));
      CHK(hipGraphDestroy(g));
    }
    for (int w = 0; w < 2; ++w)
      for (int p = 0; p < S; ++p) CHK(hipGraphLaunch(ex[p], st[p]));
    CHK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(e0, st[0]));
      for (int p = 1; p < S; ++p) CHK(hipStreamWaitEvent(st[p], e0, 0));
      for (int p = 0; p < S; ++p) CHK(hipGraphLaunch(ex[p], st[p]));
      for (int p = 1; p < S; ++p) {
        CHK(hipEventRecord(done[p], st[p]));
        CHK(hipStreamWaitEvent(st[0], done[p], 0));
      }
      CHK(hipEventRecord(e1, st[0]));
      CHK(hipEventSynchronize(e1));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      const double per = ms / K;
      printf("{\"pattern\": \"the step, one graph per stream\", \"lds_fwd\": %d, \"lds_inv\": %d, \"stagger\": %lld, "
             "\"streams\": %d, \"rep\": %d, \"ms_per_step\": %.4f, \"Msamples_per_s\": %.1f, \"GBps\": %.1f}\n", lds_f,
             lds_i, pstr - plane, S, rep, per,
             plane / (per * 1e-3) / 1e6, step_bytes / (per * 1e-3) / 1e9);
      fflush(stdout);
    }
    for (auto& x : ex) CHK(hipGraphExecDestroy(x));
  };
  for (int S : {1, 2, 4, 8}) run_graph(S);
  if (argc > 2 && argc <= 4) return 0;
  for (int S : {1, smax}) {
    run("fwd sc1 stores + inv nt (the step)", S, [&](const Set& s, long long rows, long long r0, hipStream_t q) {
      hipLaunchKernelGGL(fanout<16>, dim3((unsigned)rows), dim3(512), 0, q, s.x, s.c, N, pstr, J, r0);
    });
    run("fwd nt stores + inv nt", S, [&](const Set& s, long long rows, long long r0, hipStream_t q) {
      hipLaunchKernelGGL(fanout<-1>, dim3((unsigned)rows), dim3(512), 0, q, s.x, s.c, N, pstr, J, r0);
    });
    run("fwd write-back stores + inv nt", S, [&](const Set& s, long long rows, long long r0, hipStream_t q) {
      hipLaunchKernelGGL(fanout<0>, dim3((unsigned)rows), dim3(512), 0, q, s.x, s.c, N, pstr, J, r0);
    });
  }
  // each pass alone (1 stream, rotated sets): the forward pattern, then the inverse pattern
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = 0; i < WARM; ++i) {
      const Set& s = sets[i % R];
      if (pass == 0) hipLaunchKernelGGL(fanout<16>, dim3(B), dim3(512), 0, st[0], s.x, s.c, N, pstr, J, 0LL);
      else hipLaunchKernelGGL(fanin, dim3(B), dim3(512), 0, st[0], s.c, s.y, N, pstr, J, 0LL);
    }
    CHK(hipEventRecord(e0, st[0]));
    for (int i = 0; i < K; ++i) {
      const Set& s = sets[i % R];
      if (pass == 0) hipLaunchKernelGGL(fanout<16>, dim3(B), dim3(512), 0, st[0], s.x, s.c, N, pstr, J, 0LL);
      else hipLaunchKernelGGL(fanin, dim3(B), dim3(512), 0, st[0], s.c, s.y, N, pstr, J, 0LL);
    }
    CHK(hipEventRecord(e1, st[0]));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"pattern\": \"%s alone\", \"ms_per_launch\": %.4f, \"GBps\": %.1f}\n", pass ? "inverse 7->1 nt" : "forward 1->7 sc1",
           ms / K, plane * 64.0 / (ms / K * 1e-3) / 1e9);
    fflush(stdout);
  }
  return 0;
}
