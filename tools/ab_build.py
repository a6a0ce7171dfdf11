"""Build a development variant of libnart_hip.so into abbuild/NAME (A/B timing on the GPU box,
selected there with NART_HIP_LIB=abbuild/NAME/libnart_hip.so).

    python tools/ab_build.py NAME -DNART_SPLAT_SKEW=20 [...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from nart_amd import build as b  # noqa: E402


def main(name, *defines):
    scene = b.build_scene_lib()
    out_dir = os.path.join(REPO, "abbuild", name)
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "libnart_hip.so")
    b._run([b.hipcc(), "--offload-arch=" + b.ARCH, "-fhip-fp32-correctly-rounded-divide-sqrt"] + b.COMMON +
           list(defines) + ["-shared", "-o", out, os.path.join(b.CSRC, "render.hip"),
                            os.path.join(b.CSRC, "host", "bvh_build.cpp"), "-L" + os.path.dirname(scene),
                            "-lnart_scene", "-Wl,-rpath," + b.LIB])
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
