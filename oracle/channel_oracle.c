/*
 * channel_oracle.c -- CPU restatement of the on-device synthetic frame source.
 *
 * TEST INFRASTRUCTURE ONLY (see spa_oracle.c header).  Restates the frame
 * source of csrc/spa_kernels.hip:generate_kernel, which itself reproduces the
 * reference's frame pipeline with a counter-based RNG in place of the
 * reference's time-seeded MT19937 (channel.py:30) and Python `random`
 * (generator.py:7-9) -- so parity here is with OUR generator bit for bit (bits,
 * codeword) and to the ulp of log/cos/sin (noise); parity with the reference is
 * statistical only:
 *   DataBuffer(k) info bits                 data_buffer.py:16-25, generator.py:7-9
 *   c = G^T u = [u, A u mod 2]              data_buffer.py:47-82, encoder_decoder_data.py:319-344
 *   BPSK bit0 -> -1, bit1 -> +1             channel.py:48-49
 *   y = x + sigma^2 * N(0,1)                channel.py:55-76 (std = sigma^2, on purpose)
 *   llr = 2 y / sigma^2                     channel.py:80
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void oracle_philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

static double u52(uint32_t hi, uint32_t lo) {
    const uint64_t x = (((uint64_t)hi << 32) | lo) >> 12;
    return ((double)x + 0.5) * 0x1p-52;
}

static void frame_bits(uint32_t k0, uint32_t k1, int64_t F, int snr_point, int k, uint8_t *u) {
    const uint32_t flo = (uint32_t)F, fhi = (uint32_t)((uint64_t)F >> 32);
    const int kw = (k + 31) / 32;
    for (int blk = 0; blk * 4 < kw; ++blk) {
        uint32_t w[4] = {flo, fhi, (uint32_t)blk, (uint32_t)snr_point << 1};
        oracle_philox4x32_10(w, k0, k1);
        for (int q = 0; q < 4; ++q)
            for (int b = 0; b < 32; ++b) {
                const int i = (blk * 4 + q) * 32 + b;
                if (i < k) u[i] = (uint8_t)((w[q] >> b) & 1u);
            }
    }
}

static void frame_channel(uint32_t k0, uint32_t k1, int64_t F, int snr_point, double sigma, int n, const uint8_t *c,
                          double *llr) {
    const uint32_t flo = (uint32_t)F, fhi = (uint32_t)((uint64_t)F >> 32);
    const double s2 = sigma * sigma;
    for (int jb = 0; jb < n; jb += 2) {
        uint32_t w[4] = {flo, fhi, (uint32_t)(jb >> 1), ((uint32_t)snr_point << 1) | 1u};
        oracle_philox4x32_10(w, k0, k1);
        const double u1 = u52(w[0], w[1]);
        const double u2 = u52(w[2], w[3]);
        const double r = sqrt(-2.0 * log(u1));
        const double th = 6.283185307179586 * u2;
        const double g[2] = {r * cos(th), r * sin(th)};
        for (int q = 0; q < 2 && jb + q < n; ++q) {
            const int j = jb + q;
            const double x = c[j] ? 1.0 : -1.0;
            const double y = x + s2 * g[q];
            llr[j] = (2.0 * y) / s2;
        }
    }
}

/*
 * Frames frame0..frame0+count-1 of SNR point snr_point.  H is CSR (m x n).
 * ira == 0: H_std = [A | I_m], c = [u, A u mod 2] (generate_kernel).
 * ira == 1: H = [H_info | staircase], c = [u, p], p_r = p_{r-1} ^ (H_info u)_r
 *           (csrc/ira_kernels.hip, ldpc_amd/ira.py).
 * u_out [count][k] (uint8), c_out [count][n] (uint8), llr_out [count][n]; any
 * may be NULL.  Returns 0 or -1.
 */
static int generate(int m, int n, const int *row_ptr, const int *col_idx, uint64_t seed, int snr_point,
                    double sigma, int64_t frame0, int count, int ira, uint8_t *u_out, uint8_t *c_out,
                    double *llr_out) {
    const int k = n - m;
    if (k < 0 || count < 0 || !(sigma > 0.0)) return -1;
    uint8_t *u = (uint8_t *)malloc((size_t)(k > 0 ? k : 1));
    uint8_t *c = (uint8_t *)malloc((size_t)n);
    double *l = (double *)malloc(sizeof(double) * (size_t)n);
    if (!u || !c || !l) {
        free(u);
        free(c);
        free(l);
        return -1;
    }
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int f = 0; f < count; ++f) {
        const int64_t F = frame0 + f;
        frame_bits(k0, k1, F, snr_point, k, u);
        memcpy(c, u, (size_t)k);
        uint8_t acc = 0;
        for (int r = 0; r < m; ++r) {
            uint8_t p = 0;
            for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e)
                if (col_idx[e] < k) p ^= u[col_idx[e]];
            acc = ira ? (uint8_t)(acc ^ p) : p;
            c[k + r] = acc;
        }
        frame_channel(k0, k1, F, snr_point, sigma, n, c, l);
        if (u_out && k > 0) memcpy(u_out + (size_t)f * k, u, (size_t)k);
        if (c_out) memcpy(c_out + (size_t)f * n, c, (size_t)n);
        if (llr_out) memcpy(llr_out + (size_t)f * n, l, sizeof(double) * (size_t)n);
    }
    free(u);
    free(c);
    free(l);
    return 0;
}

int oracle_generate_frames(int m, int n, const int *row_ptr, const int *col_idx, uint64_t seed,
                           int snr_point, double sigma, int64_t frame0, int count, uint8_t *u_out,
                           uint8_t *c_out, double *llr_out) {
    return generate(m, n, row_ptr, col_idx, seed, snr_point, sigma, frame0, count, 0, u_out, c_out, llr_out);
}

int oracle_ira_generate_frames(int m, int n, const int *row_ptr, const int *col_idx, uint64_t seed,
                               int snr_point, double sigma, int64_t frame0, int count, uint8_t *u_out,
                               uint8_t *c_out, double *llr_out) {
    return generate(m, n, row_ptr, col_idx, seed, snr_point, sigma, frame0, count, 1, u_out, c_out, llr_out);
}
