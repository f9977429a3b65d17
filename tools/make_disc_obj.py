#!/usr/bin/env python3
"""Writes gpu-ecs-madrona_amd/data/disc16.obj: a 16-gon prism (radius 1.2,
height 0.8) whose 16-vertex caps stress the narrowphase clip buffers."""
import math
import os

N, R, H = 16, 1.2, 0.4
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "gpu-ecs-madrona_amd", "data", "disc16.obj")


def main():
    lines = ["# 16-gon prism (disc): radius 1.2, height 0.8 (tools/make_disc_obj.py)", "o disc16"]
    for z in (-H, H):
        for i in range(N):
            a = 2 * math.pi * i / N
            lines.append(f"v {R * math.cos(a):.7f} {R * math.sin(a):.7f} {z}")
    lines.append("f " + " ".join(str(i) for i in range(N, 0, -1)))
    lines.append("f " + " ".join(str(N + i) for i in range(1, N + 1)))
    for i in range(N):
        a, b = i + 1, (i + 1) % N + 1
        lines.append(f"f {a} {b} {N + b} {N + a}")
    with open(OUT, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
