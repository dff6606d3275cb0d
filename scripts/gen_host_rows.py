"""Extract every ``[runtime]``-flavour HostPlacement row of the reference's kernel dispatch
tables (``moose/src/kernels/*.rs``, ``modelled_kernel!`` blocks) into
``tests/fixtures/host_rows.json``: ``[{"op", "args", "ret", "vararg", "src"}]``.

The rows are the reference's host leaf kernels (``moose/src/host/*.rs``); the generated
test (``tests/test_host_rows.py``) runs a one-op textual graph for each of them on the
graph executor.  Re-run after changing the reference checkout::

    python scripts/gen_host_rows.py /root/reference
"""
import glob
import json
import os
import re
import sys

_BLOCK = re.compile(r"modelled_kernel!\s*\{(.*?)\n\}", re.S)
_HDR = re.compile(r"^\s*[\w:]+\s*,\s*(\w+)Op\b")
_ROW = re.compile(r"\(HostPlacement,\s*(vec\[(\w+)\]|\(([^)]*)\))\s*->\s*(\w+)\s*=>\s*"
                  r"\[runtime\]")


def extract(ref_root):
    rows = []
    kdir = os.path.join(ref_root, "moose", "src", "kernels")
    for path in sorted(glob.glob(os.path.join(kdir, "*.rs"))):
        text = open(path).read()
        for m in _BLOCK.finditer(text):
            body = m.group(1)
            hdr = _HDR.match(body.strip())
            if hdr is None:
                continue
            op = hdr.group(1)
            line0 = text[:m.start()].count("\n") + 1
            for r in _ROW.finditer(body):
                if r.group(2) is not None:
                    args, vararg = [r.group(2)], True
                else:
                    args = [a.strip() for a in r.group(3).split(",") if a.strip()]
                    vararg = False
                line = line0 + body[:r.start()].count("\n")
                rows.append({"op": op, "args": args, "ret": r.group(4), "vararg": vararg,
                             "src": f"moose/src/kernels/{os.path.basename(path)}:{line}"})
    return rows


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    rows = extract(ref)
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(here, "tests", "fixtures", "host_rows.json")
    with open(out, "w") as f:
        json.dump(rows, f, indent=0)
        f.write("\n")
    print(f"{len(rows)} rows -> {out}")


if __name__ == "__main__":
    main()
