// Host check of the device math helpers of csrc/mpcg_device.h (fsincos) against the C
// library: the largest ulp distance over seeded uniform samples per argument range, and
// the signed zeros.  Built by tests/test_device_math.py with hipcc (host code only).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "mpcg_device.h"

static int64_t ulps(double a, double b) {
    int64_t ia, ib;
    memcpy(&ia, &a, 8);
    memcpy(&ib, &b, 8);
    if (ia < 0) ia = INT64_MIN - ia;
    if (ib < 0) ib = INT64_MIN - ib;
    return ia > ib ? ia - ib : ib - ia;
}

int main() {
    std::mt19937_64 g(7);
    const double ranges[] = {1e-6, 0.5, 3.2, 50.0, 1e4, 1e6};
    for (double R : ranges) {
        std::uniform_real_distribution<double> u(-R, R);
        int64_t ms = 0, mc = 0;
        for (int i = 0; i < 400000; ++i) {
            const double x = u(g);
            double s, c;
            mpcg::fsincos(x, &s, &c);
            const int64_t a = ulps(s, std::sin(x)), b = ulps(c, std::cos(x));
            ms = a > ms ? a : ms;
            mc = b > mc ? b : mc;
        }
        printf("range %g sin_ulp %lld cos_ulp %lld\n", R, (long long)ms, (long long)mc);
    }
    double s, c;
    mpcg::fsincos(-0.0, &s, &c);
    printf("negzero %d %g\n", std::signbit(s) ? 1 : 0, c);
    return 0;
}
