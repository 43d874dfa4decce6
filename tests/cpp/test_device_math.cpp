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
    // atan / atan2 with the host division as the reciprocal
    struct Div {
        double operator()(double d) const { return 1.0 / d; }
    };
    const double aranges[] = {1e-9, 0.3, 1.0, 3.0, 100.0, 1e20};
    for (double R : aranges) {
        std::uniform_real_distribution<double> u(-R, R);
        int64_t ma = 0, m2 = 0;
        for (int i = 0; i < 400000; ++i) {
            const double x = u(g), y = u(g);
            const int64_t a = ulps(mpcg::fatan(x, Div{}), std::atan(x));
            const int64_t b = ulps(mpcg::fatan2(y, x, Div{}), std::atan2(y, x));
            ma = a > ma ? a : ma;
            m2 = b > m2 ? b : m2;
        }
        printf("arange %g atan_ulp %lld atan2_ulp %lld\n", R, (long long)ma, (long long)m2);
    }
    printf("aspecial %.17g %.17g %.17g %.17g %.17g %d\n", mpcg::fatan2(0.0, -1.0, Div{}), mpcg::fatan2(1.0, 0.0, Div{}),
           mpcg::fatan2(-1.0, -0.0, Div{}), mpcg::fatan(1e300, Div{}), mpcg::fatan(INFINITY, Div{}),
           std::signbit(mpcg::fatan(-0.0, Div{})) ? 1 : 0);
    double s, c;
    mpcg::fsincos(-0.0, &s, &c);
    printf("negzero %d %g\n", std::signbit(s) ? 1 : 0, c);
    return 0;
}
