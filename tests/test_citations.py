"""Every `name.ext:a` / `name.ext:a-b` citation of a reference file in the sources (oracle/,
nart_amd/, include/, bench.py, tests/) points inside that file: a <= b <= its line count.  The
line counts are a fixture made from the reference (tools/make_ref_line_counts.py), so the check
runs without /root/reference.  File names the reference does not have (this repo's own files,
e.g. kernels.h, render.hip) are not citations of it; host/main.cpp cites itself as
`host/main.cpp`, so a bare `main.cpp:` is the reference's."""
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"(?<![\w/])((?:[\w.-]+/)*)([A-Za-z_][\w]*\.(?:cpp|h|py|txt|json)):(\d+)(?:-(\d+))?")
DIRS = ["oracle", "nart_amd", "include", "tests", "tools"]
FILES = ["bench.py", "__graft_entry__.py"]
OWN_PREFIXES = ("host/", "device/", "csrc/", "nart_amd/", "tests/", "tools/", "oracle/")


def sources():
    for d in DIRS:
        for root, dirs, files in os.walk(os.path.join(REPO, d)):
            dirs[:] = [x for x in dirs if x not in ("__pycache__", "_ref", "build", "golden")]
            for f in files:
                if f.endswith((".c", ".h", ".cpp", ".hip", ".py", ".sh")):
                    yield os.path.join(root, f)
    for f in FILES:
        yield os.path.join(REPO, f)


def test_reference_citations_fall_inside_the_files():
    with open(os.path.join(REPO, "tests", "golden", "ref_line_counts.json")) as fh:
        counts = json.load(fh)
    bad, seen = [], 0
    for path in sources():
        if os.path.basename(path) == "test_citations.py":
            continue
        with open(path, encoding="utf-8", errors="replace") as fh:
            for ln, line in enumerate(fh, 1):
                for m in PAT.finditer(line):
                    prefix, name, a, b = m.group(1), m.group(2), int(m.group(3)), m.group(4)
                    if name not in counts or prefix.startswith(OWN_PREFIXES):
                        continue
                    b = int(b) if b else a
                    seen += 1
                    n = counts[name]["lines"]
                    if not (1 <= a <= b <= n):
                        bad.append("%s:%d cites %s:%d-%d (file has %d lines)" % (
                            os.path.relpath(path, REPO), ln, name, a, b, n))
    assert seen > 100
    assert not bad, "\n".join(bad)
