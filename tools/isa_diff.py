"""Compare the gfx950 ISA of two device-assembly dumps kernel by kernel (hipcc -S
--cuda-device-only): prints, per kernel symbol, whether its instruction stream is identical once
labels and comments are normalised.  Used to show that a source refactor leaves the shipped
kernels' code unchanged (same instructions => same bits, same time)."""
import re
import sys


def kernels(path):
    out, cur, name = {}, None, None
    for line in open(path):
        m = re.match(r'^(_Z\S+):\s*(;.*)?$', line)
        if m:
            name, cur = m.group(1), []
            continue
        if name is None:
            continue
        if line.startswith('.Lfunc_end'):
            out[name] = cur
            name = None
            continue
        s = line.split(';')[0].strip()
        if not s or s.startswith('.'):
            continue
        s = re.sub(r'\.LBB\d+_\d+', 'L', s)
        cur.append(s)
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    for n in sorted(set(a) | set(b)):
        if n not in a or n not in b:
            print(f"{'only-before' if n in a else 'only-after ':11s} {n}")
            continue
        same = a[n] == b[n]
        print(f"{'same' if same else 'DIFF':11s} {n} ({len(a[n])} -> {len(b[n])} instrs)")


if __name__ == '__main__':
    main()
