"""Generate tests/golden/dumpR3_frames.npz from the reference's own trajectory file.

Source (read-only, only present in the build container):
  /root/reference/CUDA-Parallel-MC/CUDA-Parallel-MC/dumpR3.txt
  -- 1000 frames of 64 atoms written by create_dump (kernel.cu:510-536), LAMMPS text format,
     box [-5, 5]^3 (L = 10), coordinates printed with %f.

Stored vectors (data only; no reference source is copied):
  frame_ids          the frame indices kept (0, 1, 2, 500, 999)
  positions[k]       float64 (64, 3) coordinates of frame frame_ids[k] as printed
  energy_calc[k]     total LJ energy of that frame with the reference's host energy function
                     calc_energy (kernel.cu:452-470): minimum image |d| > L/2 -> |d| - L, r <= rc
                     (rc = 2.5), 4(r^-12 - r^-6), evaluated here in float64
  max_occupancy[k]   largest cell count of the frame binned into the 4^3 grid (w = 2.5) with the
                     reference's assign rule lb < x <= ub (start.cu:129-134)
  frame_text_0/1     the exact bytes of frames 0 and 1 as create_dump printed them (uint8) -- the
                     golden output of the dump writer (pmc_write_dump) and the reader's input

Run:  python tests/golden/make_golden.py
"""
import os

import numpy as np

SRC = "/root/reference/CUDA-Parallel-MC/CUDA-Parallel-MC/dumpR3.txt"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dumpR3_frames.npz")
KEEP = (0, 1, 2, 500, 999)
L, RC, W, CPS = 10.0, 2.5, 2.5, 4


def parse_frames(path):
    frames = []
    with open(path) as f:
        lines = f.read().splitlines()
    i = 0
    while i < len(lines):
        if lines[i].startswith("ITEM: TIMESTEP"):
            natoms = int(lines[i + 3])
            atoms = lines[i + 9:i + 9 + natoms]
            pos = np.array([[float(t) for t in a.split()[2:5]] for a in atoms], np.float64)
            frames.append(pos)
            i += 9 + natoms
        else:
            i += 1
    return frames


def calc_energy(pos):
    e = 0.0
    n = len(pos)
    for i in range(n):
        d = np.abs(pos[i + 1:] - pos[i])
        d = np.where(d > L / 2, d - L, d)
        r = np.sqrt((d * d).sum(1))
        r = r[r <= RC]
        p6 = r ** -6.0
        e += float(np.sum(4.0 * (p6 * p6 - p6)))
    return e


def max_occ(pos):
    cnt = {}
    for x in pos:
        idx = []
        for v in x:
            c = int(np.ceil((v + L / 2) / W)) - 1   # lb < v <= ub
            idx.append(min(max(c, 0), CPS - 1))
        cnt[tuple(idx)] = cnt.get(tuple(idx), 0) + 1
    return max(cnt.values())


def frame_texts(path, count):
    """Raw bytes of the first `count` frames (each starts at an 'ITEM: TIMESTEP' line)."""
    data = open(path, "rb").read()
    starts = []
    pos = 0
    while len(starts) <= count:
        i = data.find(b"ITEM: TIMESTEP", pos)
        if i < 0:
            break
        starts.append(i)
        pos = i + 1
    return [np.frombuffer(data[starts[k]:starts[k + 1]], np.uint8) for k in range(count)]


def main():
    frames = parse_frames(SRC)
    texts = frame_texts(SRC, 2)
    assert len(frames) == 1000, len(frames)
    pos = np.stack([frames[k] for k in KEEP])
    en = np.array([calc_energy(frames[k]) for k in KEEP])
    occ = np.array([max_occ(frames[k]) for k in KEEP])
    np.savez_compressed(OUT, frame_ids=np.array(KEEP), positions=pos, energy_calc=en, max_occupancy=occ,
                        frame_text_0=texts[0], frame_text_1=texts[1])
    print(OUT, en, occ)


if __name__ == "__main__":
    main()
