#!/usr/bin/env python3
"""Writes gpu-ecs-madrona_amd/data/disc{N}.obj: an N-gon prism (radius 1.2,
height 0.8) whose N-vertex caps stress the narrowphase clip buffers.
disc16 (N = 16) fits the contact kernel's LDS clip buffers; disc64 does not
(2 x 64 vertices x 28 B x 128 lanes = 458 KB > 160 KB), so its worlds run the
global-image contact and SAT kernels."""
import math
import os
import sys

R, H = 1.2, 0.4
DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "gpu-ecs-madrona_amd", "data")


def write(n):
    name = f"disc{n}"
    lines = [f"# {n}-gon prism (disc): radius 1.2, height 0.8 (tools/make_disc_obj.py)", f"o {name}"]
    for z in (-H, H):
        for i in range(n):
            a = 2 * math.pi * i / n
            lines.append(f"v {R * math.cos(a):.7f} {R * math.sin(a):.7f} {z}")
    lines.append("f " + " ".join(str(i) for i in range(n, 0, -1)))
    lines.append("f " + " ".join(str(n + i) for i in range(1, n + 1)))
    for i in range(n):
        a, b = i + 1, (i + 1) % n + 1
        lines.append(f"f {a} {b} {n + b} {n + a}")
    with open(os.path.join(DATA, name + ".obj"), "w") as f:
        f.write("\n".join(lines) + "\n")


def main():
    for n in (int(x) for x in (sys.argv[1:] or ["16", "64"])):
        write(n)


if __name__ == "__main__":
    main()
