"""The reference's stdout contract, byte for byte.

    cintegrate   "%lf seconds\\n"  +  "final distance is:%lf\\n"        cintegrate.cu:140-141
    riemann      "%lf seconds\\n"  +  cout.precision(15) sentence         riemann.cpp:92-96
    4main        "Step size of %ld\\n", "%lf seconds\\n",
                 "Total distance traveled = %lf\\n"                        4main.c:73,239,241
"""
from __future__ import annotations


def fmt_seconds(s: float) -> str:
    return "%f seconds" % s


def fmt_cintegrate_distance(d: float) -> str:
    return "final distance is:%f" % d


def cpp_precision15(x: float) -> str:
    """std::ostream with precision(15) in default float format (== printf %.15g)."""
    return "%.15g" % x


def fmt_riemann_result(b: float, n: float, g_sum: float) -> str:
    return ("The integral of f(x) from 0.0 to " + cpp_precision15(b) + " with "
            + cpp_precision15(n) + " steps is " + cpp_precision15(g_sum))


def fmt_step_size(steps_per_sec: int) -> str:
    return "Step size of %d" % steps_per_sec


def fmt_total_distance(d: float) -> str:
    return "Total distance traveled = %f" % d
