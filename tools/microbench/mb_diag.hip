// Microbenchmark of k_ldlt_t16's diagonal-tile factorization (t16_diag): cycles per call.
#include "../../orb-slam3-noted_amd/csrc/lba.hip"

#include <cstdio>
#include <cstring>

struct DiagLds {
    double D[256];
    double M[kT16Max][16 * kPStride];
    double dinv[kT16Max][16];
    double y[kT16Max * 16];
    double wb[2][16];
    int fail;
};

__global__ void k_bench(const double* A, double* out, long long* cyc, int reps) {
    __shared__ DiagLds L;
    const int lane = threadIdx.x;
    if (lane < 16) L.y[lane] = 1.0;
    L.fail = 0;
    double4_t dt = *(const double4_t*)(A + 4 * lane);
    const long long t0 = wall_clock64();
    for (int r = 0; r < reps; r++) {
        t16_diag(L, r & 1, dt, lane);
        dt[0] += L.M[r & 1][lane & 15] * 1e-30;  // keep the calls dependent
    }
    const long long t1 = wall_clock64();
    out[lane] = L.M[0][lane] + L.M[0][64 + lane] + L.M[0][128 + lane] + L.M[0][192 + lane] + L.dinv[0][lane & 15] + L.y[lane & 15];
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    // SPD 16x16 in the transposed accumulator layout (symmetric: the tile itself)
    double Ah[256], A[256];
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) Ah[i * 16 + j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
    for (int l = 0; l < 64; l++)
        for (int u = 0; u < 4; u++) A[4 * l + u] = Ah[(l & 15) * 16 + (l >> 4) + 4 * u];
    double *dA, *dO;
    long long* dc;
    hipMalloc(&dA, sizeof(A));
    hipMalloc(&dO, 64 * sizeof(double));
    hipMalloc(&dc, sizeof(long long));
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    const int reps = 200;
    k_bench<<<1, 64>>>(dA, dO, dc, reps);
    k_bench<<<1, 64>>>(dA, dO, dc, reps);
    long long c;
    hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    printf("t16_diag: %.2f us per call (wall clock 100 MHz)\n", c / 100.0 / reps);
    // one call's outputs (M_0, 1/d, z_0) for comparing the variants bit for bit
    k_bench<<<1, 64>>>(dA, dO, dc, 1);
    double o[64];
    hipMemcpy(o, dO, sizeof(o), hipMemcpyDeviceToHost);
    unsigned long long h = 1469598103934665603ull;
    for (int l = 0; l < 64; l++) {
        unsigned long long b;
        memcpy(&b, &o[l], 8);
        h = (h ^ b) * 1099511628211ull;
    }
    printf("outputs fnv %016llx  o[0] %.17g o[17] %.17g o[63] %.17g\n", h, o[0], o[17], o[63]);
    return 0;
}
