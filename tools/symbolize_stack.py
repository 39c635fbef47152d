"""Map the raw addresses of a glog-style crash stack ("@ 0x7f… (unknown)") to library + offset using a
/proc/<pid>/maps dump of the same process (tools/exit_probe.py writes one), then ask llvm-symbolizer for
the function.  The libraries are this image's, so the symbolisation can run in the build container.

    python tools/symbolize_stack.py STACK_LOG MAPS
"""
import re
import subprocess
import sys

SYMBOLIZER = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def load_maps(path):
    rows = []
    for line in open(path):
        f = line.split()
        if len(f) < 6:
            continue
        lo, hi = (int(x, 16) for x in f[0].split("-"))
        rows.append((lo, hi, int(f[2], 16), f[5]))
    return rows


def locate(maps, addr):
    for lo, hi, off, name in maps:
        if lo <= addr < hi:
            return name, addr - lo + off
    return None, None


def main():
    stack, maps_path = sys.argv[1], sys.argv[2]
    maps = load_maps(maps_path)
    addrs = [int(m, 16) for m in re.findall(r"@\s+0x([0-9a-f]+)", open(stack).read())]
    fault = re.search(r"SIGSEGV \(@0x([0-9a-f]+)\)", open(stack).read())
    if fault:
        name, off = locate(maps, int(fault.group(1), 16))
        print(f"fault address 0x{fault.group(1)} -> {name or 'UNMAPPED at exit-time dump'} +0x{off or 0:x}")
    for a in addrs:
        name, off = locate(maps, a)
        sym = ""
        if name and name.startswith("/"):
            try:
                sym = subprocess.run([SYMBOLIZER, "--obj", name, f"0x{off:x}"], capture_output=True, text=True,
                                     timeout=30).stdout.split("\n")[0]
            except Exception as e:  # noqa: BLE001
                sym = f"({e})"
        print(f"0x{a:x}  {name}+0x{(off or 0):x}  {sym}")


if __name__ == "__main__":
    main()
