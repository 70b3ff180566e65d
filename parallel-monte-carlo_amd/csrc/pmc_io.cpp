// pmc_io.cpp -- trajectory dump / restart: host-only C ABI functions
// declared in include/pmc.h.  No HIP here: these run (and are tested) without a GPU; the
// context-level wrappers (pmc_dump_frame, pmc_save_snapshot, pmc_load_snapshot) in pmc_api.hip copy
// the device state out/in and call them.
//
// Reference: disk_to_r and create_dump (CUDA-Parallel-MC/CUDA-Parallel-MC/kernel.cu:497-536), the
// host-side visualisation path of the reference's main loop (kernel.cu:622-627, 688-701), which
// writes LAMMPS-style text frames for OVITO.  The reference has no reader and no checkpoint; the
// reader and the binary snapshot (exact float bits + the sweep counter, which is the whole RNG
// state of the counter-based Philox streams) are this build's restart path.
#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pmc.h"

extern "C" int pmc_io_fail(int code, const char* msg);   // pmc_api.hip: sets pmc_last_error()
static int pmc_io_fail(int code, const std::string& msg) { return pmc_io_fail(code, msg.c_str()); }

namespace {

constexpr char kMagic[8] = {'P', 'M', 'C', 'S', 'N', 'A', 'P', '1'};
constexpr uint32_t kVersion = 1;
constexpr uint32_t kHeaderBytes = 160;

// FNV-1a 64 over the payload bytes (integrity check of a snapshot)
struct Fnv {
    uint64_t h = 1469598103934665603ull;
    void add(const void* p, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) {
            h ^= b[i];
            h *= 1099511628211ull;
        }
    }
};

template <class T>
void put(unsigned char* buf, size_t off, T v) { std::memcpy(buf + off, &v, sizeof(T)); }
template <class T>
T get(const unsigned char* buf, size_t off) {
    T v;
    std::memcpy(&v, buf + off, sizeof(T));
    return v;
}

// header field offsets (bytes)
enum : size_t {
    H_MAGIC = 0, H_VERSION = 8, H_HBYTES = 12, H_INTS = 16 /* 8 x i32: cps_x..n_moves */,
    H_W = 48, H_BETA = 52, H_SIGMA = 56, H_FLAGS = 60, H_SEED = 64, H_SWEEP = 72,
    H_STATS = 80 /* 4 x i64 */, H_CELLS = 112, H_ATOMS = 120, H_SUM = 128
};

struct File {
    FILE* f = nullptr;
    explicit File(FILE* ff) : f(ff) {}
    ~File() {
        if (f) std::fclose(f);
    }
};

}  // namespace

extern "C" {

int pmc_disk_to_r(const float* h_disk, const int16_t* h_n, int64_t cells, int32_t nmax, float* h_r,
                  int64_t stride, int64_t* count) {
    if (!h_disk || !h_n || cells < 0 || nmax <= 0 || stride < 0) return pmc_io_fail(PMC_ERR_ARG, "pmc_disk_to_r: bad argument");
    int64_t k = 0;
    for (int64_t c = 0; c < cells; ++c) {
        const int m = h_n[c];
        if (m < 0 || m > nmax) return pmc_io_fail(PMC_ERR_ARG, "pmc_disk_to_r: cell count outside [0, nmax]");
        if (h_r && k + m > stride) return pmc_io_fail(PMC_ERR_ARG, "pmc_disk_to_r: more particles than stride");
        if (h_r) {
            const float* row = h_disk + (size_t)c * 3 * (size_t)nmax;
            for (int j = 0; j < m; ++j)                      // kernel.cu:503-508: cell, then slot
                for (int dim = 0; dim < 3; ++dim) h_r[(size_t)stride * dim + (size_t)(k + j)] = row[(size_t)dim * nmax + j];
        }
        k += m;
    }
    if (count) *count = k;
    return PMC_OK;
}

int pmc_write_dump(const char* path, int append, int64_t timestep, const float* h_r, int64_t stride,
                   int64_t n_atoms, const float box_lo[3], const float box_hi[3]) {
    if (!path || (n_atoms > 0 && !h_r) || n_atoms < 0 || stride < n_atoms || !box_lo || !box_hi)
        return pmc_io_fail(PMC_ERR_ARG, "pmc_write_dump: bad argument");
    // the stdio buffer must outlive the stream (fclose flushes from it): declared first
    std::vector<char> buf(1 << 20);
    // append by seeking to the end of an "r+" stream (not O_APPEND, whose semantics some
    // network / overlay file systems do not honour); a missing file is created
    File fp(append ? std::fopen(path, "r+") : nullptr);
    if (!fp.f) fp.f = std::fopen(path, "w");
    if (!fp.f) return pmc_io_fail(PMC_ERR_ARG, std::string("pmc_write_dump: cannot open ") + path + ": " + std::strerror(errno));
    if (append && std::fseek(fp.f, 0, SEEK_END) != 0) return pmc_io_fail(PMC_ERR_ARG, "pmc_write_dump: seek failed");
    std::setvbuf(fp.f, buf.data(), _IOFBF, buf.size());
    // create_dump, kernel.cu:521-535 (the reference prints %i; identical text for < 2^31 atoms)
    std::fprintf(fp.f,
                 "ITEM: TIMESTEP \n%" PRId64 "\nITEM: NUMBER OF ATOMS\n%" PRId64
                 "\nITEM: BOX BOUNDS\n%f %f\n%f %f\n%f %f\nITEM: ATOMS id type x y z ix iy iz\n",
                 timestep, n_atoms, (double)box_lo[0], (double)box_hi[0], (double)box_lo[1], (double)box_hi[1],
                 (double)box_lo[2], (double)box_hi[2]);
    for (int64_t j = 0; j < n_atoms; ++j)
        std::fprintf(fp.f, "%" PRId64 " %" PRId64 " %f %f %f 0 0 0\n", j + 1, j + 1, (double)h_r[j],
                     (double)h_r[(size_t)stride + (size_t)j], (double)h_r[2 * (size_t)stride + (size_t)j]);
    if (std::ferror(fp.f)) return pmc_io_fail(PMC_ERR_ARG, "pmc_write_dump: write error");
    return PMC_OK;
}

int pmc_read_dump(const char* path, int64_t frame, int64_t* timestep, float* h_r, int64_t stride,
                  int64_t* n_atoms, float box_lo[3], float box_hi[3]) {
    if (!path || frame < 0) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: bad argument");
    File fp(std::fopen(path, "r"));
    if (!fp.f) return pmc_io_fail(PMC_ERR_ARG, std::string("pmc_read_dump: cannot open ") + path + ": " + std::strerror(errno));
    std::vector<char> line(4096);
    auto next = [&]() -> bool { return std::fgets(line.data(), (int)line.size(), fp.f) != nullptr; };
    auto starts = [&](const char* s) { return std::strncmp(line.data(), s, std::strlen(s)) == 0; };
    int64_t seen = -1;
    while (next()) {
        if (!starts("ITEM: TIMESTEP")) continue;
        ++seen;
        if (!next()) break;
        const int64_t ts = std::strtoll(line.data(), nullptr, 10);
        if (!next() || !starts("ITEM: NUMBER OF ATOMS") || !next()) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: malformed frame header");
        const int64_t na = std::strtoll(line.data(), nullptr, 10);
        if (!next() || !starts("ITEM: BOX BOUNDS")) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: malformed frame header");
        float lo[3], hi[3];
        for (int d = 0; d < 3; ++d) {
            if (!next()) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: truncated box bounds");
            char* e = nullptr;
            lo[d] = std::strtof(line.data(), &e);
            hi[d] = std::strtof(e, nullptr);
        }
        if (!next() || !starts("ITEM: ATOMS")) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: malformed frame header");
        if (seen < frame) {                      // skip this frame's atom lines
            for (int64_t j = 0; j < na; ++j)
                if (!next()) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: truncated frame");
            continue;
        }
        if (timestep) *timestep = ts;
        if (n_atoms) *n_atoms = na;
        if (box_lo) std::memcpy(box_lo, lo, sizeof(lo));
        if (box_hi) std::memcpy(box_hi, hi, sizeof(hi));
        if (!h_r) return PMC_OK;
        if (stride < na) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: stride smaller than the frame's atom count");
        for (int64_t j = 0; j < na; ++j) {
            if (!next()) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: truncated frame");
            char* p = line.data();
            char* e = nullptr;
            const int64_t id = std::strtoll(p, &e, 10);   // atoms are placed by id (1-based)
            p = e;
            (void)std::strtoll(p, &e, 10);                // type
            p = e;
            if (id < 1 || id > na) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: atom id out of range");
            for (int d = 0; d < 3; ++d) {
                h_r[(size_t)stride * d + (size_t)(id - 1)] = std::strtof(p, &e);
                if (e == p) return pmc_io_fail(PMC_ERR_ARG, "pmc_read_dump: malformed atom line");
                p = e;
            }
        }
        return PMC_OK;
    }
    return pmc_io_fail(PMC_ERR_RANGE, "pmc_read_dump: frame not found");
}

int pmc_snapshot_write(const char* path, const pmc_params* p, uint32_t next_sweep, const pmc_stats* st,
                       const float* h_disk, const int16_t* h_n, int64_t cells) {
    if (!path || !p || !h_disk || !h_n || cells < 0) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_write: bad argument");
    const int nm = p->nmax;
    // payload: counts, then per cell its occupied slots x[0..n), y[0..n), z[0..n) (exact bits)
    std::vector<unsigned char> pay((size_t)cells * 2);
    std::memcpy(pay.data(), h_n, (size_t)cells * 2);
    int64_t atoms = 0;
    for (int64_t c = 0; c < cells; ++c) {
        if (h_n[c] < 0 || h_n[c] > nm) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_write: cell count outside [0, nmax]");
        atoms += h_n[c];
    }
    const size_t coord0 = pay.size();
    pay.resize(coord0 + (size_t)atoms * 12);
    size_t o = coord0;
    for (int64_t c = 0; c < cells; ++c) {
        const int m = h_n[c];
        const float* row = h_disk + (size_t)c * 3 * (size_t)nm;
        for (int d = 0; d < 3; ++d) {
            std::memcpy(pay.data() + o, row + (size_t)d * nm, (size_t)m * 4);
            o += (size_t)m * 4;
        }
    }
    Fnv sum;
    sum.add(pay.data(), pay.size());
    unsigned char h[kHeaderBytes];
    std::memset(h, 0, sizeof(h));
    std::memcpy(h + H_MAGIC, kMagic, 8);
    put<uint32_t>(h, H_VERSION, kVersion);
    put<uint32_t>(h, H_HBYTES, kHeaderBytes);
    const int32_t ints[8] = {p->cps_x, p->cps_y, p->cps_z, p->nz_local, p->z0, p->halo, p->nmax, p->n_moves};
    std::memcpy(h + H_INTS, ints, sizeof(ints));
    put<float>(h, H_W, p->w);
    put<float>(h, H_BETA, p->beta);
    put<float>(h, H_SIGMA, p->sigma);
    put<uint32_t>(h, H_FLAGS, p->flags);
    put<uint64_t>(h, H_SEED, p->seed);
    put<uint32_t>(h, H_SWEEP, next_sweep);
    const int64_t s4[4] = {st ? st->de_fixed : 0, st ? st->accepted : 0, st ? st->trials : 0, st ? st->evaluated : 0};
    std::memcpy(h + H_STATS, s4, sizeof(s4));
    put<int64_t>(h, H_CELLS, cells);
    put<int64_t>(h, H_ATOMS, atoms);
    put<uint64_t>(h, H_SUM, sum.h);
    // write to path.tmp, then rename: a crash never leaves a half-written snapshot under path
    const std::string tmp = std::string(path) + ".tmp";
    {
        File fp(std::fopen(tmp.c_str(), "wb"));
        if (!fp.f) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_write: cannot open " + tmp + ": " + std::strerror(errno));
        if (std::fwrite(h, 1, sizeof(h), fp.f) != sizeof(h) ||
            std::fwrite(pay.data(), 1, pay.size(), fp.f) != pay.size() || std::fflush(fp.f) != 0)
            return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_write: write error");
    }
    if (std::rename(tmp.c_str(), path) != 0) return pmc_io_fail(PMC_ERR_ARG, std::string("pmc_snapshot_write: rename: ") + std::strerror(errno));
    return PMC_OK;
}

int pmc_snapshot_read(const char* path, pmc_params* p, uint32_t* next_sweep, pmc_stats* st, float* h_disk,
                      int16_t* h_n, int64_t cells) {
    if (!path) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: bad argument");
    File fp(std::fopen(path, "rb"));
    if (!fp.f) return pmc_io_fail(PMC_ERR_ARG, std::string("pmc_snapshot_read: cannot open ") + path + ": " + std::strerror(errno));
    unsigned char h[kHeaderBytes];
    if (std::fread(h, 1, sizeof(h), fp.f) != sizeof(h) || std::memcmp(h + H_MAGIC, kMagic, 8) != 0)
        return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: not a PMCSNAP1 file");
    if (get<uint32_t>(h, H_VERSION) != kVersion || get<uint32_t>(h, H_HBYTES) != kHeaderBytes)
        return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: unsupported snapshot version");
    pmc_params q;
    std::memset(&q, 0, sizeof(q));
    int32_t ints[8];
    std::memcpy(ints, h + H_INTS, sizeof(ints));
    q.cps_x = ints[0]; q.cps_y = ints[1]; q.cps_z = ints[2]; q.nz_local = ints[3];
    q.z0 = ints[4]; q.halo = ints[5]; q.nmax = ints[6]; q.n_moves = ints[7];
    q.w = get<float>(h, H_W);
    q.beta = get<float>(h, H_BETA);
    q.sigma = get<float>(h, H_SIGMA);
    q.flags = get<uint32_t>(h, H_FLAGS);
    q.seed = get<uint64_t>(h, H_SEED);
    const int64_t fcells = get<int64_t>(h, H_CELLS), atoms = get<int64_t>(h, H_ATOMS);
    // the caller's buffers hold `cells` rows of 3*p->nmax floats: refuse any other nmax before
    // writing anything (p is input here, the snapshot's parameters on return)
    if ((h_disk || h_n) && (!p || p->nmax != q.nmax))
        return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: snapshot nmax differs from the buffer's (params->nmax)");
    if (p) *p = q;
    if (next_sweep) *next_sweep = get<uint32_t>(h, H_SWEEP);
    if (st) {
        int64_t s4[4];
        std::memcpy(s4, h + H_STATS, sizeof(s4));
        st->de_fixed = s4[0]; st->accepted = s4[1]; st->trials = s4[2]; st->evaluated = s4[3];
    }
    if (!h_disk && !h_n) return PMC_OK;                       // header only
    if (!h_disk || !h_n || cells != fcells) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: cell count differs from the snapshot");
    if (fcells < 0 || atoms < 0 || q.nmax <= 0) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: corrupt header");
    std::vector<unsigned char> pay((size_t)fcells * 2 + (size_t)atoms * 12);
    if (std::fread(pay.data(), 1, pay.size(), fp.f) != pay.size()) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: truncated payload");
    Fnv sum;
    sum.add(pay.data(), pay.size());
    if (sum.h != get<uint64_t>(h, H_SUM)) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: checksum mismatch");
    const int nm = q.nmax;
    std::memcpy(h_n, pay.data(), (size_t)fcells * 2);
    std::memset(h_disk, 0, (size_t)fcells * 3 * (size_t)nm * 4);
    size_t o = (size_t)fcells * 2;
    int64_t k = 0;
    for (int64_t c = 0; c < fcells; ++c) {
        const int m = h_n[c];
        if (m < 0 || m > nm || (k += m) > atoms) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: corrupt counts");
        float* row = h_disk + (size_t)c * 3 * (size_t)nm;
        for (int d = 0; d < 3; ++d) {
            std::memcpy(row + (size_t)d * nm, pay.data() + o, (size_t)m * 4);
            o += (size_t)m * 4;
        }
    }
    if (k != atoms) return pmc_io_fail(PMC_ERR_ARG, "pmc_snapshot_read: corrupt counts");
    return PMC_OK;
}

}  // extern "C"
