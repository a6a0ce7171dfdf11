"""In-tree build of the nart_amd native libraries (no CMake, no network).

    libnart_scene.so  host ingestion / CLI params / EXR I/O (g++, no HIP)
    libnart_hip.so    gfx950 render path + C ABI (hipcc --offload-arch=gfx950)
    nart              CLI drop-in for the reference's `nart <scene> <out> [flags]`

Every translation unit is compiled with -ffp-contract=off: the render path reproduces the
reference's float arithmetic bit for bit, so no multiply-add may be fused.
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
LIB = os.path.join(ROOT, "lib")
BIN = os.path.join(ROOT, "bin")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"

COMMON = ["-std=c++17", "-O3", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-result",
          "-Wno-unused-value", "-Wno-unused-function"]


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def _newer(target, sources):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(s) <= t for s in sources)


def _sources(*rel):
    out = []
    for r in rel:
        p = os.path.join(CSRC, r)
        if os.path.isdir(p):
            out += [os.path.join(p, f) for f in sorted(os.listdir(p)) if f.endswith((".h", ".hip", ".cpp"))]
        else:
            out.append(p)
    return out


def hip_source_sha():
    """sha256 (16 hex digits) of the sources of libnart_hip.so: ties a committed profile (e.g.
    profiles/pmc_latest.json's HBM traffic) to the kernel code it was measured on."""
    import hashlib
    h = hashlib.sha256()
    for f in _sources("render.hip", "device", "host/bvh_build.cpp", "host/bvh_build.h", "host/multi_gpu.h"):
        h.update(os.path.relpath(f, CSRC).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_scene_lib(force=False):
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, "libnart_scene.so")
    srcs = _sources("host/scene_host.cpp", "host/json.h", "host/exr_piz.cpp", "host/exr_piz.h") + \
        [os.path.join(REPO, "include", "nart_scene.h")]
    if not force and _newer(out, srcs):
        return out
    _run(["g++"] + COMMON + ["-shared", "-o", out, os.path.join(CSRC, "host", "scene_host.cpp"),
                             os.path.join(CSRC, "host", "exr_piz.cpp"), "-lz"])
    return out


def hipcc():
    return shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def build_hip_lib(force=False):
    scene = build_scene_lib()
    out = os.path.join(LIB, "libnart_hip.so")
    srcs = _sources("render.hip", "device", "host") + [os.path.join(REPO, "include", "nart_hip.h"), scene]
    if not force and _newer(out, srcs):
        return out
    extra = os.environ.get("NART_HIP_DEFINES", "").split()  # development builds, e.g. -DNART_WAVEPROF
    # -fno-slp-vectorize: no packed-f32 pairs (v_pk_mul_f32 ...) -- their aligned register pairs
    # raised the ray-queue kernel's register peak (C3 build 230 -> 207 VGPRs without them); the
    # same IEEE operations either way
    _run([hipcc(), "--offload-arch=" + ARCH, "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize"] +
         COMMON + extra +
         ["-shared", "-o", out, os.path.join(CSRC, "render.hip"), os.path.join(CSRC, "host", "bvh_build.cpp"),
          "-L" + LIB, "-lnart_scene", "-Wl,-rpath,$ORIGIN"])
    return out


def build_cli(force=False):
    hip = build_hip_lib()
    os.makedirs(BIN, exist_ok=True)
    out = os.path.join(BIN, "nart")
    src = os.path.join(CSRC, "host", "main.cpp")
    if not force and _newer(out, [src, hip]):
        return out
    _run(["g++"] + COMMON + ["-o", out, src, "-L" + LIB, "-lnart_hip", "-lnart_scene",
                             "-Wl,-rpath,$ORIGIN/../lib"])
    return out


def build_all(force=False):
    build_scene_lib(force)
    build_hip_lib(force)
    build_cli(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
