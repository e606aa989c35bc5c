"""Slot-update count of the register LDL^T for cyclic lane layouts.

A wave's 64 lanes hold an n x n lower triangle as a PR x QC lane grid (PR * QC = 64): lane
(p, q) of slot (r, s) holds element (PR r + p, QC s + q).  Column step k updates every slot
(r, s) that holds a live trailing element: slot columns s with a column > k, slot rows from the
one holding row QC s down.  Each slot update is one FMA instruction per lane, whatever part of
the slot is live -- the count below is the factorisation's FMA instructions per lane (before
the persistent kernel's pivot / publication work), against the perfect distribution of the
(n - k)(n - k - 1) / 2 trailing updates of step k over 64 lanes.

    python tools/layout_model.py [n]
"""
import sys


def slot_updates(pr: int, qc: int, n: int) -> int:
    total = 0
    for k in range(n):
        for s in range((k + 1) // qc, n // qc):
            total += n // pr - (qc * s) // pr
    return total


def ideal(n: int) -> float:
    return sum((n - k) * (n - k - 1) / 2 / 64 for k in range(n))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    print(f"n = {n}: ideal {ideal(n):.0f} FMA instructions per lane")
    for pr, qc in ((8, 8), (16, 4), (4, 16), (32, 2)):
        print(f"  {pr:2d} x {qc:2d} lanes: {slot_updates(pr, qc, n)}")


if __name__ == "__main__":
    main()
