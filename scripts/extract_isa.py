"""Disassemble the gfx950 code object inside a hipcc object / shared library (its clang offload bundle):
    python scripts/extract_isa.py <file.o|.so> <out.s>"""
import struct
import subprocess
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path):
    d = open(path, "rb").read()
    pos = d.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", d, pos + 24)[0]
        off = pos + 32
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", d, off)
            triple = d[off + 24: off + 24 + tl].decode()
            off += 24 + tl
            if "gfx" in triple:
                yield triple, d[pos + o: pos + o + sz]
        pos = d.find(MAGIC, pos + 1)


if __name__ == "__main__":
    src, out = sys.argv[1], sys.argv[2]
    for k, (triple, co) in enumerate(code_objects(src)):
        tmp = f"{out}.{k}.co"
        open(tmp, "wb").write(co)
        with open(out if k == 0 else f"{out}.{k}", "w") as f:
            subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--symbolize-operands", tmp], stdout=f, check=True)
        print(triple, len(co))
