"""Register / scratch / LDS figures of every kernel in libcmpc.so's gfx950 code objects (the AMDGPU metadata notes
that llvm-readelf --notes prints), one row per kernel: the .hip_fatbin section is dumped with llvm-objcopy, each
translation unit's clang offload bundle is split out, and its gfx950 code object is read with llvm-readelf --notes.
Usage: python tools/co_notes.py [lib] > profiles/<round>_libcmpc_notes.txt"""
import hashlib
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(lib):
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")],
                       check=True)
        data = open(fb, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        offs, i = [], data.find(magic)
        while i >= 0:
            offs.append(i)
            i = data.find(magic, i + 1)
        rows = []
        for n, o in enumerate(offs):
            nent = struct.unpack_from("<Q", data, o + 24)[0]
            p = o + 32
            for _ in range(nent):
                off, size, idl = struct.unpack_from("<QQQ", data, p)
                p += 24
                tid = data[p:p + idl].decode()
                p += idl
                if "gfx950" not in tid:
                    continue
                co = os.path.join(d, f"co_{n}.co")
                open(co, "wb").write(data[o + off:o + off + size])
                notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
                for blk in re.split(r"\n  - \.", notes):  # kernel entries (2-space indent; their args nest deeper)
                    m = re.search(r"\.name:\s+(\S+)", blk)
                    if not m or ".vgpr_count" not in blk:
                        continue

                    def g(key):
                        mm = re.search(r"(?:^|\n)\s*\.?" + key + r":\s+(\d+)", blk)
                        return int(mm.group(1)) if mm else -1
                    rows.append((m.group(1), g("vgpr_count"), g("agpr_count"), g("sgpr_count"), g("vgpr_spill_count"),
                                 g("sgpr_spill_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size")))
        return rows


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), "cheeta-mpc_amd", "lib", "libcmpc.so")
    rows = kernels(lib)
    names = [r[0] for r in rows]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    md5 = hashlib.md5(open(lib, "rb").read()).hexdigest()
    print(f"# llvm-readelf --notes of {os.path.basename(lib)} (md5 {md5}), gfx950 code objects: {len(rows)} kernels")
    print("# vgpr = .vgpr_count, agpr = .agpr_count (the notes' own fields); spills = .vgpr_spill_count /")
    print("# .sgpr_spill_count; rocprofv3's VGPR_Count column is not this count (it reads 128 for k_solve64<double, 2>")
    print("# at 253 here, 256 for k_ocp_grid at 436 / 180: profiles/r05_sq_*.txt 'resources')")
    print("# (SGPR spills go to VGPR lanes, not to memory); scratch = .private_segment_fixed_size bytes; lds = static")
    print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'vspill':>6} {'sspill':>6} {'scratch':>7} {'lds':>6}  kernel")
    for r, dn in sorted(zip(rows, dem), key=lambda t: t[1]):
        print(f"{r[1]:>5} {r[2]:>5} {r[3]:>5} {r[4]:>6} {r[5]:>6} {r[6]:>7} {r[7]:>6}  {dn}")


if __name__ == "__main__":
    main()
