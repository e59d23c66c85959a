// What it costs to hand a value from one wavefront of a workgroup to another and back -- the step a
// trajectory split over two waves (VERDICT r02 "Next round" 3: a partner wave computing the BDF
// coefficients / eta candidates / dense output while the first runs the Newton chain) would pay per
// exchange. One workgroup of two waves (normally on two SIMDs of one CU); wave 0 writes a double to
// LDS, wave 1 reads it, adds 1, writes it back, wave 0 reads it: one round trip.
//   mode 0: __syncthreads (s_barrier) between the writes and the reads (two barriers per trip)
//   mode 1: LDS flags: the reader spins on a sequence number (no barrier; spins bounded)
//   mode 2: reference: the same add done by wave 0 alone (dependent f64 add chain)
// Prints cycles (clock64) per round trip.
//   hipcc -O3 --offload-arch=gfx950 -o build/handoff handoff.hip && ./build/handoff
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int TRIPS = 2048;

template <int MODE>
__global__ void __launch_bounds__(128) handoff(double* out, long long* cyc)
{
    __shared__ double box[2];
    __shared__ volatile int seq[2];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) {
        box[0] = box[1] = 0.0;
        seq[0] = seq[1] = 0;
    }
    __syncthreads();
    double v = 1.0;
    const long long t0 = clock64();
    for (int t = 0; t < TRIPS; t++) {
        if constexpr (MODE == 0) {
            if (wave == 0 && lane == 0) box[0] = v;
            __syncthreads();
            if (wave == 1) {
                const double x = box[0] + 1.0;
                if (lane == 0) box[1] = x;
            }
            __syncthreads();
            if (wave == 0) v = box[1];
        } else if constexpr (MODE == 1) {
            if (wave == 0) {
                if (lane == 0) {
                    box[0] = v;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    seq[0] = t + 1;
                }
                for (int spin = 0; spin < (1 << 16) && seq[1] != t + 1; spin++) {
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                v = box[1];
            } else {
                for (int spin = 0; spin < (1 << 16) && seq[0] != t + 1; spin++) {
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const double x = box[0] + 1.0;
                if (lane == 0) {
                    box[1] = x;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    seq[1] = t + 1;
                }
            }
        } else {
            if (wave == 0) {
                v = v + 1.0;
                asm volatile("" : "+v"(v));
            }
        }
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) {
        out[0] = v;
        cyc[0] = t1 - t0;
    }
}

template <int MODE>
static void run(const char* name)
{
    double* dout;
    long long* dcyc;
    hipMalloc(&dout, sizeof(double));
    hipMalloc(&dcyc, sizeof(long long));
    long long best = -1;
    double v = 0.0;
    for (int rep = 0; rep < 5; rep++) {
        hipLaunchKernelGGL(handoff<MODE>, dim3(1), dim3(128), 0, 0, dout, dcyc);
        hipDeviceSynchronize();
        long long c;
        hipMemcpy(&c, dcyc, sizeof(c), hipMemcpyDeviceToHost);
        hipMemcpy(&v, dout, sizeof(v), hipMemcpyDeviceToHost);
        if (best < 0 || c < best) best = c;
    }
    printf("%-34s %8.1f clock64 ticks per round trip (value %.0f)\n", name, (double)best / TRIPS, v);
    hipFree(dout);
    hipFree(dcyc);
}

int main()
{
    run<0>("two waves, LDS + s_barrier x2");
    run<1>("two waves, LDS + sequence flags");
    run<2>("one wave, dependent f64 add");
    return 0;
}
