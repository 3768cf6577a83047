"""Fold the raw per-run bench lines of an A/B directory (NAME.R.json, one
JSON line each, written by profiles/ab.sh / ab_opts.sh) into one
DIR/runs.json {"NAME.R": line, ...}; the summaries (DIR.txt, LOG.md) cite the
directory, and profiles/ab_report_kernels.py reads runs.json as it read the
files.  Keeps profiles/ under a few hundred tracked files.

    python profiles/fold_runs.py profiles/r4/subq [more dirs]   (or --all)
"""
import glob
import json
import os
import re
import sys

RUN = re.compile(r"^(.+)\.(\d+)\.json$")


def fold(d):
    runs = {}
    files = sorted(glob.glob(os.path.join(d, "*.json")))
    for f in files:
        m = RUN.match(os.path.basename(f))
        if not m:
            continue
        text = open(f).read().strip()
        try:
            runs[m.group(1) + "." + m.group(2)] = json.loads(text.splitlines()[-1]) if text else None
        except (ValueError, IndexError):
            runs[m.group(1) + "." + m.group(2)] = {"raw": text}
    if not runs:
        return 0
    out = os.path.join(d, "runs.json")
    old = json.load(open(out)) if os.path.exists(out) else {}
    old.update(runs)
    with open(out, "w") as fh:
        json.dump(old, fh, indent=0, sort_keys=True)
    n = 0
    for f in files:
        if RUN.match(os.path.basename(f)):
            os.remove(f)
            n += 1
    return n


def main():
    dirs = sys.argv[1:]
    if dirs == ["--all"]:
        root = os.path.dirname(os.path.abspath(__file__))
        dirs = sorted({os.path.dirname(f) for f in glob.glob(os.path.join(root, "**", "*.json"), recursive=True)
                       if RUN.match(os.path.basename(f))})
    total = 0
    for d in dirs:
        n = fold(d)
        total += n
        if n:
            print("%s: %d runs folded" % (os.path.relpath(d), n))
    print("total", total)


if __name__ == "__main__":
    main()
