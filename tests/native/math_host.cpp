// Host build of the decoder's device math (ldpc-simulator_amd/csrc/spa_math.h)
// so tests/test_math.py can check, on the CPU, the exact code the kernels run.
#include "../../ldpc-simulator_amd/csrc/spa_math.h"

extern "C" void host_np_tanh(const double *x, double *y, long n) {
    ldpc::HostTanhTab t;
    for (long i = 0; i < n; ++i) y[i] = ldpc::np_tanh(x[i], t);
}
extern "C" void host_atanh(const double *x, double *y, long n) {
    ldpc::HostAtanhTab t;
    for (long i = 0; i < n; ++i) y[i] = ldpc::atanh_f(x[i], t);
}
extern "C" void host_log(const double *x, double *y, long n) {
    ldpc::HostLogTab t;
    for (long i = 0; i < n; ++i) {
        double h, l;
        ldpc::log_hilo(x[i], t, h, l);
        y[i] = h + l;
    }
}
extern "C" void host_tanh_half_clipped(const double *m, double *y, long n) {
    ldpc::HostTanhTab t;
    for (long i = 0; i < n; ++i) y[i] = ldpc::tanh_half_clipped(m[i], t);
}
