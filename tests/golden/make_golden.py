"""Generate tests/golden/shp_known_answers.json.

The fixtures are the INPUTS and EXPECTED OUTPUTS of the reference's own
tests for the hot path, recomputed here with plain Python/numpy (independent
of oracle/oracle.c, so the oracle can be checked against them):

  ShpTests.Iota / ForEach / ReduceBasic   test/gtest/shp/algorithms.cpp:11-59
  ShpTests.InclusiveScan                  test/gtest/shp/algorithms.cpp:61-149
      inputs: the unseeded glibc lrand48() % 100 stream (glibc zero-initialises
      the drand48 state; the test never calls srand48), 6 blocks of 100;
      expected: std::inclusive_scan (the test's own oracle) in wrapping int32.
  MhpTests.Reduce                         test/gtest/mhp/algorithms.cpp:124-135
  MhpTests.Stencil                        test/gtest/mhp/stencil.cpp:15-55
  examples/mhp/stencil-1d.cpp check()     examples/mhp/stencil-1d.cpp:21-45

Run: python tests/golden/make_golden.py   (writes the JSON next to itself)
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


class Lrand48:
    """glibc lrand48: X' = (0x5DEECE66D * X + 0xB) mod 2^48, result X' >> 17."""

    def __init__(self, x=0):
        self.x = x

    def __call__(self):
        self.x = (0x5DEECE66D * self.x + 0xB) & ((1 << 48) - 1)
        return self.x >> 17


def wrap32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


def inclusive_scan(xs, op, init=None):
    out, acc = [], None
    for i, x in enumerate(xs):
        if i == 0:
            acc = x if init is None else (init + x if op == "plus" else init * x)
        else:
            acc = acc + x if op == "plus" else acc * x
        acc = wrap32(acc)
        out.append(acc)
    return out


def main():
    g = {}
    # ---- ShpTests.Iota: iota from 20 over n = 10
    g["iota"] = {"n": 10, "start": 20, "expected": list(range(20, 30))}
    # ---- ShpTests.ForEach: iota 100, negate
    g["for_each_negate"] = {"n": 10, "start": 100, "expected": [-v for v in range(100, 110)]}
    # ---- ShpTests.ReduceBasic: iota 10 over n = 10, init 0, plus
    g["reduce_basic"] = {"n": 10, "start": 10, "init": 0, "expected": sum(range(10, 20))}
    # ---- ShpTests.InclusiveScan
    rng = Lrand48(0)
    layout = [("plus", None, "inplace"), ("plus", None, "misaligned"), ("mul", 12, "misaligned"),
              ("plus", None, "inplace"), ("plus", None, "misaligned"), ("mul", 12, "misaligned")]
    blocks = []
    for op, init, lay in layout:
        xs = [rng() % 100 for _ in range(100)]
        blocks.append({"op": op, "init": init, "layout": lay, "input": xs,
                       "expected": inclusive_scan(xs, op, init)})
    g["inclusive_scan"] = {"n": 100, "out_size": 200, "blocks": blocks}
    # ---- MhpTests.Reduce: iota 100 over n = 10 -> 1045
    g["mhp_reduce"] = {"n": 10, "start": 100, "init": 0, "expected": sum(range(100, 110))}
    # ---- MhpTests.Stencil: radius 4, s = v + sum_{i=0..r}(p[-i] + p[i])
    n, r = 10, 4
    vin = list(range(10, 10 + n))
    vout = [100] * n
    for i in range(r, n - r):
        s = vin[i]
        for k in range(r + 1):
            s += vin[i - k] + vin[i + k]
        vout[i] = s
    g["mhp_stencil"] = {"n": n, "radius": r, "in_start": 10, "out_fill": 100, "expected": vout}
    # ---- stencil-1d example: n = 10, 5 steps, 3-point, fixed ends
    n, steps = 10, 5
    a = list(range(100, 100 + n))
    b = [0] * n
    cur, nxt = a, b
    for _ in range(steps):
        for i in range(1, n - 1):
            nxt[i] = cur[i - 1] + cur[i] + cur[i + 1]
        cur, nxt = nxt, cur
    g["stencil_1d"] = {"n": n, "steps": steps, "a_start": 100, "b_fill": 0,
                       "expected_interior": cur[1:n - 1]}
    path = os.path.join(HERE, "shp_known_answers.json")
    with open(path, "w") as f:
        json.dump(g, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
