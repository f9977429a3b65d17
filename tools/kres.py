#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of one HIP source, from
the compiler's kernel-resource-usage remarks (device pass only, no GPU).

    python tools/kres.py gpu-ecs-madrona_amd/csrc/envs/fvs.hip [--src-root DIR] [-D...]

Used to A/B a source change's register cost before spending GPU time."""
import os
import re
import subprocess
import sys

FLAGS = ["-std=c++20", "-O3", "-fPIC", "--offload-arch=gfx950", "-mcode-object-version=5",
         "-ffp-contract=off", "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-x", "hip", "-c", "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage",
         "-o", "/dev/null"]


def short(name, width):
    # the kernel's name and the node / world function it instantiates, read
    # from the mangled name (c++filt gives up on the longest ones)
    k = re.search(r"\d+(\w+?(?:Kernel|Entry))I", name)
    fn = re.search(r"\d+(\w+?(?:System|Kernel|Entry|Fn))E", name[k.end():] if k else name)
    return ((k.group(1) if k else name[:40]) + (" " + fn.group(1) if fn else ""))[:width]


def main():
    args = sys.argv[1:]
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "gpu-ecs-madrona_amd")
    if "--src-root" in args:
        i = args.index("--src-root")
        root = args[i + 1]
        del args[i:i + 2]
    src = [a for a in args if not a.startswith("-")]
    extra = [a for a in args if a.startswith("-")]
    out = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + ["-I", os.path.join(root, "include"),
                         "-I", os.path.join(root, "..", "include")] + extra + src,
                         capture_output=True, text=True, cwd=root)
    rows, cur = [], None
    for line in out.stderr.splitlines():
        if "remark:" not in line:
            continue
        body = line.split("remark: ", 1)[1].split(" [-Rpass")[0].strip()
        k, _, v = body.partition(": ")
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        n = r["name"]
        print(f"{short(n, 70):70s} vgpr {r.get('VGPRs', '?'):>4} scratch "
              f"{r.get('ScratchSize [bytes/lane]', '?'):>5} occ {r.get('Occupancy [waves/SIMD]', '?'):>2} "
              f"lds {r.get('LDS Size [bytes/block]', '?')}")
    if out.returncode != 0:
        sys.stderr.write(out.stderr[-3000:])
        sys.exit(out.returncode)


if __name__ == "__main__":
    main()
