"""Line counts of the reference's source files, by base name (no two share one), for the citation
check in tests/test_citations.py: tests/golden/ref_line_counts.json.  Run in the build container,
where /root/reference exists (the GPU box has no reference):  python tools/make_ref_line_counts.py"""
import json
import os

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "ref_line_counts.json")


def main():
    counts = {}
    for root, dirs, files in os.walk(REF):
        dirs[:] = [d for d in dirs if d != ".git"]
        for f in files:
            if f.endswith((".cpp", ".h", ".py", ".txt", ".json")):
                with open(os.path.join(root, f), "rb") as fh:
                    n = len(fh.read().splitlines())
                rel = os.path.relpath(os.path.join(root, f), REF)
                assert f not in counts, ("duplicate base name", f, rel)
                counts[f] = {"path": rel, "lines": n}
    with open(OUT, "w") as fh:
        json.dump(dict(sorted(counts.items())), fh, indent=0, sort_keys=True)
    print(len(counts), "files ->", OUT)


if __name__ == "__main__":
    main()
