#!/usr/bin/env python3
"""Merge TunableOp result files into the committed table: later files win per GEMM key."""
import sys


def main():
    dst, srcs = sys.argv[1], sys.argv[2:]
    header, rows = [], {}
    for f in [dst] + srcs:
        for line in open(f):
            line = line.rstrip("\n")
            if not line:
                continue
            parts = line.split(",")
            if parts[0] == "Validator":
                if f == dst:
                    header.append(line)
                continue
            rows[(parts[0], parts[1])] = line
    with open(dst, "w") as fp:
        fp.write("\n".join(header + list(rows.values())) + "\n")
    print(f"{dst}: {len(rows)} GEMM entries")


if __name__ == "__main__":
    main()
