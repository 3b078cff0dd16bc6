// Accuracy of the hardware v_rsq_f64 / v_rcp_f64 estimates against correctly rounded host
// values (max error in ulps over random inputs); decides how many Newton steps the Cholesky
// pivot chain needs.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const double* x, double* rs, double* rc, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { rs[i] = __builtin_amdgcn_rsq(x[i]); rc[i] = __builtin_amdgcn_rcp(x[i]); }
}

static double ulps(double got, double ref) {
    return std::fabs(got - ref) / (std::nextafter(std::fabs(ref), INFINITY) - std::fabs(ref));
}

int main() {
    const int n = 1 << 20;
    std::vector<double> x(n), rs(n), rc(n);
    unsigned long long s = 7;
    for (int i = 0; i < n; ++i) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        double u = ((s >> 11) * 0x1.0p-53);
        x[i] = std::ldexp(1.0 + u, (int)(s % 80) - 40);
    }
    double *dx, *drs, *drc;
    hipMalloc(&dx, 8 * n); hipMalloc(&drs, 8 * n); hipMalloc(&drc, 8 * n);
    hipMemcpy(dx, x.data(), 8 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, drs, drc, n);
    hipMemcpy(rs.data(), drs, 8 * n, hipMemcpyDeviceToHost);
    hipMemcpy(rc.data(), drc, 8 * n, hipMemcpyDeviceToHost);
    double mrs = 0, mrc = 0;
    for (int i = 0; i < n; ++i) {
        long double r1 = 1.0L / sqrtl((long double)x[i]);
        long double r2 = 1.0L / (long double)x[i];
        mrs = std::fmax(mrs, ulps(rs[i], (double)r1));
        mrc = std::fmax(mrc, ulps(rc[i], (double)r2));
    }
    printf("{\"rsq_f64_max_ulp\": %.3g, \"rcp_f64_max_ulp\": %.3g}\n", mrs, mrc);
    return 0;
}
