"""Where a path-kernel build's VGPR pressure comes from (no GPU needed).

Compiles one instantiation of `k_render_rq` (kernels.h) with the library's flags plus line tables,
stops LLVM after the machine scheduler, runs the AMDGPU register-pressure printer
(`llc -run-pass=amdgpu-print-rp`) over that MIR and maps each instruction's VGPR pressure back to
the innermost source function and line of its debug location.  Prints the peak, the per-function
maxima (which function's live state sets the floor) and the source lines at the top of the curve.

    python tools/reg_pressure.py                        # lean glassSphere build (FM_GLASS, WV 3)
    python tools/reg_pressure.py --fm 33 --wv 3         # lean Cornell build
    python tools/reg_pressure.py --fm 1023 --wv 2 --pr  # generic two-wave build with priority lanes

Pressure is counted in 32-bit registers before allocation; the allocator's final count
(tools/kernel_regs.sh) can sit a few registers above it (alignment of 64/128-bit tuples).
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from nart_amd import build  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"
FLAGS = ["--offload-arch=gfx950", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize",
         "-std=c++17", "-O3", "-ffp-contract=off", "-fno-fast-math"]


def compile_rp(fm, wv, pr, ext, env, work):
    src = os.path.join(work, "probe.hip")
    with open(src, "w") as f:
        f.write('#include "device/kernels.h"\n'
                "template __global__ void nd::k_render_rq<%s, false, %s, %du, %d, %s>(nd::DScene, nd::RenderArgs);\n"
                % ("true" if ext else "false", "true" if env else "false", fm, wv, "true" if pr else "false"))
    bc, mir = os.path.join(work, "probe.bc"), os.path.join(work, "probe.mir")
    subprocess.run([build.hipcc()] + FLAGS + ["-I" + build.CSRC, "-I" + os.path.join(REPO, "include"),
                    "-gline-tables-only", "--cuda-device-only", "-emit-llvm", "-c", src, "-o", bc], check=True, cwd=work)
    subprocess.run([LLVM + "/llc", "-march=amdgcn", "-mcpu=gfx950", "-O3", bc, "-stop-after=machine-scheduler",
                    "-o", mir], check=True)
    rp = subprocess.run([LLVM + "/llc", "-march=amdgcn", "-mcpu=gfx950", "-run-pass=amdgpu-print-rp", mir,
                         "-o", os.devnull], capture_output=True, text=True)
    if rp.returncode:
        raise SystemExit(rp.stderr[-2000:])
    return rp.stderr


FUNC = re.compile(r"^(?:ND|NHD|__global__|__device__|static|inline)\b[^;=]*?\b(\w+)\s*(?:<[^;]*>)?\s*\(|"
                  r"^\s+(?:const\s+)?auto\s+(\w+)\s*=\s*\[")
_src = {}


def enclosing(path, line):
    """Name of the function (or named lambda) whose definition precedes `line` in `path`."""
    if path not in _src:
        try:
            _src[path] = open(path).read().splitlines()
        except OSError:
            _src[path] = []
    lines = _src[path]
    end = min(line, len(lines))
    for i in range(end - 1, -1, -1):
        m = FUNC.match(lines[i])
        if not m:
            continue
        depth, opened = 0, False  # is the definition still open at `line`?  (braces outside // comments)
        for j in range(i, end):
            code = lines[j].split("//")[0]
            for ch in code:
                if ch == "{":
                    depth, opened = depth + 1, True
                elif ch == "}":
                    depth -= 1
            if opened and depth <= 0 and j < end - 1:
                break
        else:
            k = re.search(r"\bvoid\s+(\w+)\s*\(", lines[i])  # kernels: skip __launch_bounds__(...)
            return k.group(1) if k else m.group(1) or m.group(2)
    return "?"


def text(path, line):
    lines = _src.get(path) or []
    return lines[line - 1].strip()[:64] if 0 < line <= len(lines) else ""


def frames(comment):
    """'a.h:3:1 @[ b.h:9:2 @[ c.h:1:1 ] ]' -> [(a.h, 3), (b.h, 9), (c.h, 1)] innermost first."""
    out = []
    for tok in comment.replace("]", " ").split("@["):
        m = re.match(r"\s*(\S+):(\d+):\d+", tok)
        if m:
            out.append((os.path.normpath(m.group(1)), int(m.group(2))))
    return out


def live_in(sect, fn_name):
    """VGPR state live into the block of `fn_name` (the traversal for trav_step) with the most of it,
    grouped by the source statement that defined it."""
    defs, blocks, cur = {}, {}, None
    dre = re.compile(r"^\s+\d+\s+\d+\s+(?:undef |early-clobber )*%(\d+)(?:\.\w+)?:(\w+)\b.*?;\s*(\S.*)$")
    for ln in sect.splitlines():
        b = re.match(r"^  (bb\.\d+)", ln)
        if b:
            cur = blocks.setdefault(b.group(1), {"n": 0, "in": ""})
            continue
        if cur is None:
            continue
        if ln.strip().startswith("Live-in:"):
            cur["in"] = ln
        m = dre.match(ln)
        if m:
            fr = [f for f in frames(m.group(3)) if f[0].startswith(REPO)]
            if fr and m.group(1) not in defs:
                defs[m.group(1)] = (m.group(2), fr[0], fr[-1])
            if fr and enclosing(*fr[0]) == fn_name:
                cur["n"] += 1
    vcls = ("vgpr", "vreg", "av")

    def vgprs(blk):
        out = []
        for vr, mask in re.findall(r"%(\d+):([0-9A-F]+)", blk["in"]):
            cls, inner, outer = defs.get(vr, ("?", ("?", 0), ("?", 0)))
            if cls.startswith(vcls):
                out.append((bin(int(mask, 16)).count("1") // 2, inner, outer))
        return out

    cand = [(sum(r for r, _, _ in vgprs(b)), k, b) for k, b in blocks.items() if b["n"]]
    if not cand:
        return None
    total, name, blk = max(cand, key=lambda c: c[0])
    groups = collections.defaultdict(int)
    for regs, inner, outer in vgprs(blk):
        groups[(os.path.relpath(outer[0], REPO), outer[1], enclosing(*inner))] += regs
    return name, blk["n"], total, groups


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--fm", type=int, default=37, help="feature mask (path.h FT_*; 37 glassSphere, 33 Cornell, "
                                                        "913 C4, 1023 generic)")
    ap.add_argument("--wv", type=int, default=3, help="waves per SIMD of the build (3 = lean)")
    ap.add_argument("--pr", action="store_true", help="priority lanes and speculative pairs compiled in")
    ap.add_argument("--ext", action="store_true", help="dielectric lists longer than 10 (EXT)")
    ap.add_argument("--env", action="store_true", help="environment light (ENV)")
    ap.add_argument("--through", default="trav_step", help="list the VGPR state live into this function's "
                                                             "block with the most of it")
    ap.add_argument("--top", type=int, default=25, help="source lines listed")
    ap.add_argument("--above", type=int, default=0, help="list lines whose pressure reaches this (default: peak-24)")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as work:
        rp = compile_rp(a.fm, a.wv, a.pr, a.ext, a.env, work)
    sect = [b for b in re.split(r"^name: ", rp, flags=re.M) if b.startswith("_ZN2nd11k_render_rq")]
    if len(sect) != 1:
        raise SystemExit("k_render_rq not found in the pressure printout")
    inst = re.compile(r"^\s+(\d+)\s+(\d+)\s+\S.*?;\s*(\S.*)$")
    per_fn = collections.defaultdict(lambda: [0, 0])  # innermost function -> [max vgpr, instructions]
    per_line = collections.defaultdict(int)            # (file, line, function) -> max vgpr
    per_site = collections.defaultdict(lambda: [0, 0])  # outermost call site in the kernel -> [max, count]
    peak, peak_at, n = 0, None, 0
    for ln in sect[0].splitlines():
        m = inst.match(ln)
        if not m:
            continue
        v = int(m.group(2))
        fr = [f for f in frames(m.group(3)) if f[0].startswith(REPO)] or [("?", 0)]
        path, line = fr[0]
        loc = (os.path.relpath(path, REPO) if path != "?" else "?", line, enclosing(path, line))
        n += 1
        f = per_fn[loc[2]]
        f[0], f[1] = max(f[0], v), f[1] + 1
        per_line[loc] = max(per_line[loc], v)
        op, ol = fr[-1]
        site = per_site[(os.path.relpath(op, REPO) if op != "?" else "?", ol, enclosing(op, ol))]
        site[0], site[1] = max(site[0], v), site[1] + 1
        if v > peak:
            peak, peak_at = v, loc
    print("k_render_rq<EXT=%d, COUNT=0, ENV=%d, FM=%d, WV=%d, PR=%d>: %d instructions, VGPR pressure peak %d at "
          "%s:%d (%s)" % (a.ext, a.env, a.fm, a.wv, a.pr, n, peak, *peak_at))
    print("\nper innermost source function (max VGPR pressure over its instructions, instruction count):")
    for fn, (v, c) in sorted(per_fn.items(), key=lambda kv: -kv[1][0]):
        print("  %4d  %6d  %s" % (v, c, fn))
    print("\nper statement of the kernel body (outermost frame) at pressure >= %d:" % (a.above or peak - 24))
    for (fil, line, fn), (v, c) in sorted(per_site.items(), key=lambda kv: (-kv[1][0], kv[0][1]))[:a.top]:
        if v >= (a.above or peak - 24):
            print("  %4d  %6d  %s:%d  %-16s %s" % (v, c, fil, line, fn, text(os.path.join(REPO, fil), line)))
    lt = live_in(sect[0], a.through) if a.through else None
    if lt:
        name, cnt, total, groups = lt
        print("\nVGPRs live into %s (%d of %s's instructions; the most of its blocks): %d, by defining statement:" % (name, cnt, a.through,
                                                                                          total))
        for (fil, line, fn), r in sorted(groups.items(), key=lambda kv: (-kv[1], kv[0][1]))[:a.top]:
            print("  %4d  %s:%d  %-16s %s" % (r, fil, line, fn, text(os.path.join(REPO, fil), line)))
    lim = a.above or peak - 24
    print("\nsource lines at pressure >= %d:" % lim)
    rows = sorted(((v, k) for k, v in per_line.items() if v >= lim), key=lambda r: (-r[0], r[1]))
    for v, (fil, line, fn) in rows[:a.top]:
        print("  %4d  %s:%d  %-16s %s" % (v, fil, line, fn, text(os.path.join(REPO, fil), line)))


if __name__ == "__main__":
    main()
