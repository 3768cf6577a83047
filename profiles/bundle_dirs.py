"""Bundle the measurement files of finished rounds' evidence directories into
one DIR/bundle.json per directory ({file name: text}), keeping profiles/
under ~650 tracked files.  Scripts (.sh, .py, .hip), patches
and Markdown stay as files; a directory with fewer than 3 data files is left
as it is.  LOG.md / README.md citations of DIR/FILE then name an entry of
DIR/bundle.json.

    python profiles/bundle_dirs.py profiles/r2 profiles/r3 ...     (bundle)
    python profiles/bundle_dirs.py --extract profiles/r3/g4        (restore the files)
"""
import json
import os
import sys

KEEP = (".sh", ".py", ".hip", ".patch", ".md", ".so")
DATA = (".txt", ".json", ".csv", ".log")


def bundle(d):
    for root, _dirs, files in os.walk(d):
        data = sorted(f for f in files if f.endswith(DATA) and f != "bundle.json" and not f.endswith(KEEP))
        if len(data) < 3:
            continue
        path = os.path.join(root, "bundle.json")
        b = json.load(open(path)) if os.path.exists(path) else {}
        for f in data:
            with open(os.path.join(root, f), errors="replace") as fh:
                b[f] = fh.read()
        with open(path, "w") as fh:
            json.dump(b, fh, indent=0, sort_keys=True)
        for f in data:
            os.remove(os.path.join(root, f))
        print(root, len(data))


def extract(d):
    b = json.load(open(os.path.join(d, "bundle.json")))
    for f, text in b.items():
        with open(os.path.join(d, f), "w") as fh:
            fh.write(text)


if __name__ == "__main__":
    if sys.argv[1] == "--extract":
        for d in sys.argv[2:]:
            extract(d)
    else:
        for d in sys.argv[1:]:
            bundle(d)
