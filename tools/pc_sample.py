"""Developer tool: where a render kernel's issue slots go, from rocprofv3 PC sampling.

    rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
        --pc-sampling-interval 1 -d gpurun_out/pcs -o run --output-format csv -- python3 tools/prof_target.py C3 2 64
    python tools/pc_sample.py gpurun_out/pcs [KERNEL_SUBSTRING] [--disasm CODE_OBJECT]

Counts the samples per code-object offset of the kernel (Code_Object_Offset / Instruction columns of the CSV),
prints the hottest instructions and, with --disasm (a device code object built from the same source and flags,
e.g. hipcc --cuda-device-only --no-gpu-bundle-output -c rt_runtime.hip), the share of samples per 512-byte window
of the kernel's code with its instruction mix, to find the source region each window holds."""
import collections
import csv
import glob
import os
import re
import subprocess
import sys


def samples(root, kernel_sub):
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*pc_sampling*.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append(r)
    if not rows:
        sys.exit(f"no pc sampling CSV under {root}")
    keys = list(rows[0].keys())
    off_k = next((k for k in keys if "offset" in k.lower()), None)
    ins_k = next((k for k in keys if k.lower() == "instruction"), None)
    ker_k = next((k for k in keys if "kernel" in k.lower() and "name" in k.lower()), None)
    print("columns:", keys)
    cnt = collections.Counter()
    text = {}
    for r in rows:
        if kernel_sub and ker_k and kernel_sub not in r.get(ker_k, ""):
            continue
        o = r.get(off_k, "0")
        off = int(o, 16) if o.startswith("0x") else int(o or 0)
        cnt[off] += 1
        if ins_k:
            text[off] = r.get(ins_k, "")
    return cnt, text


def disasm(co, kernel_sub):
    """(offset, instruction) of the kernel's instructions in the code object's disassembly."""
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                         text=True).stdout.splitlines()
    res, inside = [], False
    for line in out:
        m = re.match(r"^([0-9a-f]+) <(.*)>:", line)
        if m:
            inside = kernel_sub in m.group(2)
            continue
        m = re.match(r"^\s+([0-9a-f]+):\s+(\S.*?)\s*(//.*)?$", line) if inside else None
        if m:
            res.append((int(m.group(1), 16), m.group(2)))
    return res


def main():
    root = sys.argv[1]
    kernel_sub = next((a for a in sys.argv[2:] if not a.startswith("--") and not os.path.exists(a)), "")
    co = sys.argv[sys.argv.index("--disasm") + 1] if "--disasm" in sys.argv else None
    cnt, text = samples(root, kernel_sub)
    total = sum(cnt.values())
    print(f"samples: {total}")
    for off, n in cnt.most_common(40):
        print(f"  {off:#08x} {100.0 * n / total:5.2f} %  {text.get(off, '')}")
    if co:  # 512-byte windows of the kernel's code, hottest first, with their instruction mix
        ins = disasm(co, kernel_sub or "persistent")
        per = collections.Counter()
        for off, n in cnt.items():
            per[off >> 9] += n
        print("hottest 512-B windows (share, start, VALU / SALU / VMEM / LDS instructions, first instructions):")
        for w, n in per.most_common(30):
            win = [t for o, t in ins if (o >> 9) == w]
            kinds = [sum(t.startswith(p) for t in win) for p in ("v_", "s_", ("global_", "buffer_", "scratch_"), "ds_")]
            print(f"  {100.0 * n / total:5.2f} %  {w << 9:#08x}  {kinds}  {' | '.join(win[:3])}")


if __name__ == "__main__":
    main()
