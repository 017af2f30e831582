#!/usr/bin/env python3
"""Instruction mix of kernels in a hipcc device assembly file (hipcc --offload-device-only -S).
usage: isa_count.py FILE.s SUBSTRING [SUBSTRING...]   (kernels whose mangled name contains all)"""
import collections
import re
import sys


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur and line.startswith("\t") and not line.strip().startswith((".", ";")) and line.strip():
            body.append(line.strip().split()[0])
        if cur and line.startswith("\t.end_amdhsa_kernel"):
            pass
    if cur:
        yield cur, body


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, body in kernels(path):
        if all(s in name for s in subs):
            c = collections.Counter(body)
            print(name[:110], "instructions:", len(body))
            for k, v in c.most_common(20):
                print(f"   {k:28s} {v}")


if __name__ == "__main__":
    main()
