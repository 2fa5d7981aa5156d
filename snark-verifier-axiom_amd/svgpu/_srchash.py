"""Hash of the sources libsvgpu.so is built from (csrc/*, include/svgpu.h, the Makefile).

The Makefile writes it next to the library (build/SOURCES.sha256) when it links; ``_lib`` checks it
at import, so a library that travels to a GPU box prebuilt is known to match the sources beside it
(a stale build fails loudly instead of testing old code).  Run as a script: prints the hash.
"""
import hashlib
import os
import sys

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files():
    csrc = os.path.join(PKG, "csrc")
    files = [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".hpp", ".cpp"))]
    files.append(os.path.join(os.path.dirname(PKG), "include", "svgpu.h"))
    files.append(os.path.join(PKG, "Makefile"))
    return sorted(files, key=lambda p: os.path.relpath(p, os.path.dirname(PKG)))


def source_hash() -> str:
    h = hashlib.sha256()
    root = os.path.dirname(PKG)
    for p in source_files():
        h.update(os.path.relpath(p, root).replace(os.sep, "/").encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


if __name__ == "__main__":
    sys.stdout.write(source_hash() + "\n")
