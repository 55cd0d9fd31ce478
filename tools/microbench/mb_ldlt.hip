// Microbenchmark of the dense LDL^T kernel (k_ldlt) on one n x n SPD system, with per-phase
// wall-clock accounting (LBA_PHASE_TIMING).  Build: see tools/microbench/Makefile.
#define LBA_PHASE_TIMING 1
#include "../../orb-slam3-noted_amd/csrc/lba.hip"

#include <cstdio>
#include <cstring>
#include <random>

// row-major lower triangle (identity-padded) -> the tile-major scratch k_ldlt_t16 reads
__global__ void k_fill_tiles(const double* A, int n, int ld, double* Ts) {
    const int T = (n + 15) >> 4;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)(16 * T) * (16 * T);
         e += (long long)gridDim.x * blockDim.x) {
        const int R = (int)(e / (16 * T)), C = (int)(e % (16 * T));
        if (C > R) continue;
        t16_put(Ts, n, R, C, R < n ? A[(long long)R * ld + C] : (R == C ? 1.0 : 0.0));
    }
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 288;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int npad = ldlt_npad(n), N = npad + 1, ld = ldlt_ld(n);
    std::mt19937_64 rng(1);
    std::normal_distribution<double> g;
    std::vector<double> M((size_t)n * n), A((size_t)N * ld, 0.0), b(n);
    for (auto& v : M) v = g(rng);
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) {
            double s = (i == j) ? n : 0.0;
            for (int k = 0; k < n; k++) s += M[(size_t)i * n + k] * M[(size_t)j * n + k] / n;
            A[(size_t)i * ld + j] = s;
        }
    for (int i = 0; i < n; i++) A[(size_t)npad * ld + i] = b[i] = g(rng);
    for (int i = n; i < npad; i++) A[(size_t)i * ld + i] = 1.0;
    WinDesc W{};
    W.n = n;
    W.ld = ld;
    W.hs_off = 0;
    WinCtl C{};
    C.need_trial = 1;
    double *dA, *dA0, *dx;
    WinDesc* dW;
    WinCtl* dC;
    hipMalloc(&dA, sizeof(double) * A.size());
    hipMalloc(&dA0, sizeof(double) * A.size());
    hipMalloc(&dx, sizeof(double) * n);
    hipMalloc(&dW, sizeof(W));
    hipMalloc(&dC, sizeof(C));
    hipMemcpy(dA0, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
    hipMemcpy(dW, &W, sizeof(W), hipMemcpyHostToDevice);
    hipMemcpy(dC, &C, sizeof(C), hipMemcpyHostToDevice);
    const size_t lds = ldlt_lds_bytes(n);
    hipFuncSetAttribute((const void*)k_ldlt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float total = 0;
    unsigned long long zero[8] = {0};
    for (int r = 0; r < reps + 1; r++) {
        hipMemcpy(dA, dA0, sizeof(double) * A.size(), hipMemcpyDeviceToDevice);
        if (r == 1) hipMemcpyToSymbol(HIP_SYMBOL(g_ldlt_phase), zero, sizeof(zero));
        hipEventRecord(e0);
        k_ldlt<<<1, 512, lds>>>(dW, dC, dA, dx);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r) total += ms;
    }
    unsigned long long ph[8];
    hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_ldlt_phase), sizeof(ph));
    std::vector<double> x(n);
    hipMemcpy(x.data(), dx, sizeof(double) * n, hipMemcpyDeviceToHost);
    double res = 0, nb = 0;
    for (int i = 0; i < n; i++) {
        double s = 0;
        for (int j = 0; j < n; j++) s += (j <= i ? A[(size_t)i * ld + j] : A[(size_t)j * ld + i]) * x[j];
        res = std::max(res, std::fabs(s - b[i]));
        nb = std::max(nb, std::fabs(b[i]));
    }
    const double us = 1e3 * total / reps;
    // the tile kernel on the same system (tile scratch, x)
    double* dT;
    hipMalloc(&dT, (size_t)t16_tiles_bytes());
    int* dErr;
    hipMalloc(&dErr, sizeof(int));
    hipMemset(dErr, 0, sizeof(int));
    float total16 = 0;
    for (int r = 0; r < reps + 1; r++) {
        if (r == 1) hipMemcpyToSymbol(HIP_SYMBOL(g_t16_phase), zero, sizeof(zero));
        k_fill_tiles<<<256, 256>>>(dA0, n, ld, dT);
        hipEventRecord(e0);
        k_ldlt_t16<<<1, kT16Waves * 64>>>(dW, dC, dA0, dT, dx, dErr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r) total16 += ms;
    }
    unsigned long long p16[8];
    hipMemcpyFromSymbol(p16, HIP_SYMBOL(g_t16_phase), sizeof(p16));
    std::vector<double> x16(n);
    hipMemcpy(x16.data(), dx, sizeof(double) * n, hipMemcpyDeviceToHost);
    double r16 = 0;
    for (int i = 0; i < n; i++) {
        double s = 0;
        for (int j = 0; j < n; j++) s += (j <= i ? A[(size_t)i * ld + j] : A[(size_t)j * ld + i]) * x16[j];
        r16 = std::max(r16, std::fabs(s - b[i]));
    }
    // the helper-assisted form (k_ldlt_t16x: one main workgroup + kT16Helpers helpers) on the same system
    double* dWg;
    T16Sync* dSync;
    hipMalloc(&dWg, (size_t)t16_tiles_bytes() * 8);
    hipMalloc(&dSync, sizeof(T16Sync) * 8);
    hipMemset(dSync, 0, sizeof(T16Sync) * 8);
    float total16x = 0;
    for (int r = 0; r < reps + 1; r++) {
        if (r == 1) hipMemcpyToSymbol(HIP_SYMBOL(g_t16_phase), zero, sizeof(zero));
        k_fill_tiles<<<256, 256>>>(dA0, n, ld, dT);
        hipEventRecord(e0);
        k_ldlt_t16x<<<8 * (1 + kT16Helpers), kT16Waves * 64>>>(1, dW, dC, dA0, dT, dWg, dSync, dx, dErr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r) total16x += ms;
    }
    unsigned long long p16x[8];
    hipMemcpyFromSymbol(p16x, HIP_SYMBOL(g_t16_phase), sizeof(p16x));
    std::vector<double> x16x(n);
    hipMemcpy(x16x.data(), dx, sizeof(double) * n, hipMemcpyDeviceToHost);
    int errw = 0;
    hipMemcpy(&errw, dErr, sizeof(int), hipMemcpyDeviceToHost);
    const bool same16x = std::memcmp(x16x.data(), x16.data(), sizeof(double) * n) == 0;
    if (n <= 16 * kT16Max)
        printf("n=%d t16x %.1f us  x %s the one-workgroup kernel's  err_word %d  phases(us): diag0 %.1f w0-wait %.1f end-wait %.1f backsolve %.1f [w0: update %.1f diag %.1f]\n",
               n, 1e3 * total16x / reps, same16x ? "bit-identical to" : "DIFFERS from", errw, p16x[1] / 100.0 / reps,
               p16x[3] / 100.0 / reps, p16x[4] / 100.0 / reps, p16x[5] / 100.0 / reps, p16x[6] / 100.0 / reps, p16x[7] / 100.0 / reps);
    if (argc > 3) {  // x of the tile kernel, for bit-for-bit comparisons between builds
        FILE* f = fopen(argv[3], "wb");
        if (f) {
            fwrite(x16.data(), sizeof(double), n, f);
            fclose(f);
        }
    }
    if (n <= 16 * kT16Max)
        printf("n=%d t16 %.1f us  residual %.3e  phases(us): diag0 %.1f w0-wait %.1f end-wait %.1f backsolve %.1f [w0: update %.1f diag %.1f trsm %.1f]\n",
               n, 1e3 * total16 / reps, r16 / (nb > 0 ? nb : 1), p16[1] / 100.0 / reps,
               p16[3] / 100.0 / reps, p16[4] / 100.0 / reps, p16[5] / 100.0 / reps, p16[6] / 100.0 / reps, p16[7] / 100.0 / reps, p16[2] / 100.0 / reps);
    // wall_clock64 runs at 100 MHz on gfx9
    printf("n=%d ldlt %.1f us  residual %.3e  phases(us): diag %.1f [load %.1f steps %.1f] rows %.1f  trailing %.1f  "
           "backsolve %.1f\n", n, us, res / nb, (ph[1] + ph[5] + ph[6]) / 100.0 / reps, ph[5] / 100.0 / reps,
           ph[6] / 100.0 / reps, ph[2] / 100.0 / reps, ph[3] / 100.0 / reps, ph[4] / 100.0 / reps);
    return 0;
}
