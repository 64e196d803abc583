"""Resource usage of libhfa's kernels (VGPR/AGPR/SGPR, spills, LDS, scratch) from the shipped code objects.
python scripts/kinfo.py [REGEX] [--dis OUT_DIR]   (CPU only; reads hubertfa_amd/_build/libhfa.so)"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_objects(lib, td):
    fat = os.path.join(td, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(td, "x")],
                   check=True, capture_output=True)
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
    for i, o in enumerate(offs):
        part, co = os.path.join(td, f"b{i}.bin"), os.path.join(td, f"b{i}.co")
        open(part, "wb").write(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"],
                           capture_output=True)
        if r.returncode == 0 and os.path.getsize(co):
            yield co


def main():
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else ".")
    dis_dir = sys.argv[sys.argv.index("--dis") + 1] if "--dis" in sys.argv else None
    lib = os.path.join(REPO, "hubertfa_amd", "_build", "libhfa.so")
    with tempfile.TemporaryDirectory() as td:
        for co in code_objects(lib, td):
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            cur = {}
            for line in notes.splitlines():
                m = re.match(r"\s+\.(\w+):\s+(.*)$", line.replace("- .", "  ."))
                if not m:
                    continue
                k, v = m.groups()
                if k == "agpr_count":
                    cur = {"agpr_count": v}
                cur[k] = v
                if k == "wavefront_size" and "name" in cur and pat.search(cur["name"]):
                    d = subprocess.run(["c++filt", cur["name"]], capture_output=True, text=True).stdout
                    print(f"{d.strip()[:120]}\n    vgpr {cur.get('vgpr_count')} agpr {cur.get('agpr_count')} "
                          f"sgpr {cur.get('sgpr_count')} spill v{cur.get('vgpr_spill_count')} "
                          f"s{cur.get('sgpr_spill_count')} lds {cur.get('group_segment_fixed_size')} "
                          f"scratch {cur.get('private_segment_fixed_size')}")
            if dis_dir:
                os.makedirs(dis_dir, exist_ok=True)
                out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True,
                                     text=True).stdout
                open(os.path.join(dis_dir, os.path.basename(co) + ".s"), "w").write(out)


if __name__ == "__main__":
    main()
