/*
 * textbook_mc.c -- an INDEPENDENT textbook Metropolis Monte Carlo of the reference's model, used
 * only to produce statistical known answers for the oracle's move chain (tests/golden/
 * known_answers.json, tools/make_known_answers.py).  Test infrastructure: nothing in the product,
 * the oracle or the bench links or calls it.
 *
 * Model (the reference's):
 *   - N Lennard-Jones particles (epsilon = sigma_LJ = 1) in a periodic cubic box of side L;
 *   - pair energy 4 (r^-12 - r^-6) for r <= rc, 0 beyond (truncated, not shifted:
 *     calculate_pair_energy, subsweep.h:90-103, with rc = w);
 *   - trial move x_i + sigma * N(0,1) per dimension (make_move, subsweep.h:60-71);
 *   - acceptance: dE < 0, else u < exp(-beta dE) (accept_move, subsweep.h:209-216).
 * Nothing else of the reference's algorithm: NO cells, NO checkerboard, NO cell-confined moves,
 * NO shiftCells -- full minimum-image interactions, every particle free to move anywhere.  The
 * checkerboard chain (cell-confined moves + random grid shifts, Anderson et al. 2013) must sample
 * the same Boltzmann distribution, so its <E> must agree with this one.
 *
 * Arithmetic in double; RNG xoshiro256** seeded by splitmix64; normals by Box-Muller.  One sweep
 * = N trial moves, particle i = 0..N-1 in order.  The energy is sampled after every sweep;
 * <E> and its standard error come from `blocks` equal block means (batch means).
 *
 *   gcc -O2 -std=c11 -o textbook_mc tools/textbook_mc.c -lm
 *   ./textbook_mc N L beta sigma rc equil_sweeps sweeps blocks seed
 * prints one JSON object: the parameters, mean, se (batch means), acceptance, block means.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t s_rng[4];

static uint64_t splitmix64(uint64_t* x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

static uint64_t next_u64(void) {
    const uint64_t r = rotl(s_rng[1] * 5, 7) * 9;
    const uint64_t t = s_rng[1] << 17;
    s_rng[2] ^= s_rng[0];
    s_rng[3] ^= s_rng[1];
    s_rng[1] ^= s_rng[2];
    s_rng[0] ^= s_rng[3];
    s_rng[2] ^= t;
    s_rng[3] = rotl(s_rng[3], 45);
    return r;
}

/* uniform in (0, 1) */
static double u01(void) { return ((double)(next_u64() >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

static double normal(void) {
    static int have = 0;
    static double spare;
    if (have) {
        have = 0;
        return spare;
    }
    const double r = sqrt(-2.0 * log(u01())), a = 6.283185307179586477 * u01();
    spare = r * sin(a);
    have = 1;
    return r * cos(a);
}

static int N;
static double L, rc2;
static double *X, *Y, *Z;

static inline double mi(double d) { return d - L * rint(d / L); }   /* minimum image */

static inline double pair(double dx, double dy, double dz) {
    const double r2 = dx * dx + dy * dy + dz * dz;
    if (r2 > rc2) return 0.0;
    const double i6 = 1.0 / (r2 * r2 * r2);
    return 4.0 * (i6 * i6 - i6);
}

/* energy of particle i at (x, y, z) with every other particle */
static double e_one(int i, double x, double y, double z) {
    double e = 0.0;
    for (int j = 0; j < N; ++j)
        if (j != i) e += pair(mi(x - X[j]), mi(y - Y[j]), mi(z - Z[j]));
    return e;
}

static double e_total(void) {
    double e = 0.0;
    for (int i = 0; i < N; ++i)
        for (int j = i + 1; j < N; ++j) e += pair(mi(X[i] - X[j]), mi(Y[i] - Y[j]), mi(Z[i] - Z[j]));
    return e;
}

int main(int argc, char** argv) {
    if (argc != 10) {
        fprintf(stderr, "usage: %s N L beta sigma rc equil_sweeps sweeps blocks seed\n", argv[0]);
        return 2;
    }
    N = atoi(argv[1]);
    L = atof(argv[2]);
    const double beta = atof(argv[3]), sigma = atof(argv[4]), rc = atof(argv[5]);
    const long equil = atol(argv[6]), sweeps = atol(argv[7]);
    const int blocks = atoi(argv[8]);
    uint64_t seed = strtoull(argv[9], NULL, 10);
    if (N < 2 || !(L > 2.0 * rc) || blocks < 2 || sweeps < blocks || sweeps % blocks) {
        fprintf(stderr, "bad arguments (need L > 2 rc, sweeps a multiple of blocks)\n");
        return 2;
    }
    rc2 = rc * rc;
    for (int k = 0; k < 4; ++k) s_rng[k] = splitmix64(&seed);
    X = malloc(sizeof(double) * N);
    Y = malloc(sizeof(double) * N);
    Z = malloc(sizeof(double) * N);
    double* bm = calloc((size_t)blocks, sizeof(double));
    /* simple-cubic start (the reference's init_r form, kernel.cu:78-89) */
    int nc = 1;
    while (nc * nc * nc < N) ++nc;
    for (int i = 0; i < N; ++i) {
        const int a = i % nc, b = (i / nc) % nc, c = i / (nc * nc);
        X[i] = L / 2.0 * (1.0 - (2.0 * a + 1.0) / nc);
        Y[i] = L / 2.0 * (1.0 - (2.0 * b + 1.0) / nc);
        Z[i] = L / 2.0 * (1.0 - (2.0 * c + 1.0) / nc);
    }
    double E = e_total();
    long acc = 0, tri = 0;
    const long per_block = sweeps / blocks;
    for (long s = -equil; s < sweeps; ++s) {
        for (int i = 0; i < N; ++i) {
            const double nx = mi(X[i] + sigma * normal());
            const double ny = mi(Y[i] + sigma * normal());
            const double nz = mi(Z[i] + sigma * normal());
            const double dE = e_one(i, nx, ny, nz) - e_one(i, X[i], Y[i], Z[i]);
            const int ok = dE < 0.0 || u01() < exp(-beta * dE);
            if (s >= 0) {
                ++tri;
                acc += ok;
            }
            if (ok) {
                X[i] = nx;
                Y[i] = ny;
                Z[i] = nz;
                E += dE;
            }
        }
        if (s >= 0) bm[s / per_block] += E;
        if (s >= 0 && (s + 1) % 10000 == 0) E = e_total();   /* drop accumulated rounding */
    }
    double mean = 0.0;
    for (int b = 0; b < blocks; ++b) {
        bm[b] /= (double)per_block;
        mean += bm[b];
    }
    mean /= blocks;
    double var = 0.0;
    for (int b = 0; b < blocks; ++b) var += (bm[b] - mean) * (bm[b] - mean);
    const double se = sqrt(var / (blocks - 1) / blocks);
    printf("{\"N\": %d, \"L\": %.17g, \"beta\": %.17g, \"sigma\": %.17g, \"rc\": %.17g, \"equil_sweeps\": %ld, "
           "\"sweeps\": %ld, \"blocks\": %d, \"seed\": %s, \"mean\": %.10f, \"se\": %.10f, \"acceptance\": %.8f, "
           "\"block_means\": [",
           N, L, beta, sigma, rc, equil, sweeps, blocks, argv[9], mean, se, (double)acc / (double)tri);
    for (int b = 0; b < blocks; ++b) printf("%s%.8f", b ? ", " : "", bm[b]);
    printf("]}\n");
    free(X);
    free(Y);
    free(Z);
    free(bm);
    return 0;
}
