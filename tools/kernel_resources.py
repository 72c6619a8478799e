"""Per-kernel register / scratch resources of the built gfx950 library, read from its code objects.

The library's .hip_fatbin section is a sequence of clang offload bundles (one per translation unit); each
holds a host stub and the gfx950 code object.  The code object's AMDGPU metadata note (llvm-readelf
--notes) lists, per kernel: .vgpr_count, .vgpr_spill_count, .sgpr_spill_count,
.private_segment_fixed_size (scratch bytes per lane), .group_segment_fixed_size (LDS).

  python tools/kernel_resources.py [lib.so] [--grep SUBSTR] [--spills]

prints one line per kernel (demangled name, VGPRs, spills, scratch, LDS).  tests/test_kernel_resources.py
uses `kernels()` to guard the hot staged kernels against scratch spills.
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "mr-vamp_amd", "vamp_amd", "libvampgpu.so")


def _fatbin(lib):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fat.bin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, out])
        with open(out, "rb") as f:
            return f.read()


def _code_objects(fat):
    """gfx950 code objects of every bundle in the section"""
    at = 0
    while True:
        at = fat.find(MAGIC, at)
        if at < 0:
            return
        p = at + len(MAGIC)
        (n,) = struct.unpack_from("<Q", fat, p)
        p += 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, p)
            p += 24
            triple = fat[p:p + tlen].decode()
            p += tlen
            if "gfx950" in triple and size:
                yield fat[at + off:at + off + size]
        at = p


_FIELDS = (".vgpr_count", ".vgpr_spill_count", ".sgpr_spill_count", ".private_segment_fixed_size",
           ".group_segment_fixed_size", ".agpr_count")


def _parse_notes(text):
    """kernel records from llvm-readelf --notes' YAML rendering of the metadata"""
    out = []
    cur = None
    for line in text.splitlines():
        # a kernel record opens with "  - .<field>:" under amdhsa.kernels; its fields sit at indent 4
        m = re.match(r"^  - (\.[a-z_]+):\s*(.*)$", line) or re.match(r"^    (\.[a-z_]+):\s*(.*)$", line)
        if not m:
            continue
        if line.startswith("  - "):
            cur = {}
            out.append(cur)
        if cur is None:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k in _FIELDS:
            cur[k] = int(v)
        elif k in (".name", ".symbol"):
            cur[k] = v
    return [k for k in out if ".symbol" in k]


def _demangle(names):
    if not names:
        return []
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        out = r.stdout.splitlines()
        return out if len(out) == len(names) else names
    except (OSError, subprocess.CalledProcessError):
        return names


def kernels(lib=DEFAULT_LIB):
    """[{name, symbol, vgpr, vgpr_spill, sgpr_spill, scratch, lds}] for every kernel of the library"""
    recs = []
    fat = _fatbin(lib)
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(_code_objects(fat)):
            path = os.path.join(d, f"co{i}.o")
            with open(path, "wb") as f:
                f.write(co)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", path], capture_output=True, text=True,
                                   check=True).stdout
            for k in _parse_notes(notes):
                recs.append({
                    "symbol": k[".symbol"].removesuffix(".kd"),
                    "vgpr": k.get(".vgpr_count", 0),
                    "vgpr_spill": k.get(".vgpr_spill_count", 0),
                    "sgpr_spill": k.get(".sgpr_spill_count", 0),
                    "scratch": k.get(".private_segment_fixed_size", 0),
                    "lds": k.get(".group_segment_fixed_size", 0),
                })
    for r, n in zip(recs, _demangle([r["symbol"] for r in recs])):
        r["name"] = n
    return recs


def main(argv):
    lib, grep, spills = DEFAULT_LIB, None, False
    it = iter(argv)
    for a in it:
        if a == "--grep":
            grep = next(it)
        elif a == "--spills":
            spills = True
        else:
            lib = a
    for r in sorted(kernels(lib), key=lambda r: r["name"]):
        if grep and grep not in r["name"]:
            continue
        if spills and not (r["scratch"] or r["vgpr_spill"]):
            continue
        print(f"{r['vgpr']:4d} vgpr {r['vgpr_spill']:4d} spill {r['scratch']:5d} B scratch {r['lds']:6d} B lds  "
              f"{r['name'][:200]}")


if __name__ == "__main__":
    main(sys.argv[1:])
