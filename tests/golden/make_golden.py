"""Writes tests/golden/reference_kat.json — the reference outputs this repo may use as fixtures.

Provenance.  The reference (erreur404/Motion-generation-using-quadratic-programs) ships no tests
and no fixtures, and its solver exists only as a prebuilt archive
(lib/QuadProgpp/libquadprog.a) that this project does not execute.  The one archive output on
record is the QuadProg++ demo problem, run by the survey and recorded in SURVEY.md §4:

    G = [[4, -2], [-2, 4]], g0 = [6, 0], CE = [1, 1]^T, ce0 = [-3],
    CI = [[1, 0, 1], [0, 1, 1]], ci0 = [0, 0, -2]   ->   f = 12, x = [1, 2.0000000000000009]

x[1] = 2.0000000000000009 is 2 + 2 ulp (0x4000000000000002): the last bits pin the operation
order of the equality step and the Givens update.  This script only transcribes those values;
it runs nothing from the reference.  The Cholesky factor of G is implied by the contract
(QuadProg++.hh:42-45) and is exact here: L = [[2, 0], [-1, sqrt(3)]] mirrored.
"""
import json
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))

kat = {
    "source": "SURVEY.md §4 (survey probe of reference lib/QuadProgpp/libquadprog.a)",
    "cases": [
        {
            "name": "quadprog_demo",
            "n": 2, "p": 1, "m": 3,
            "G": [[4.0, -2.0], [-2.0, 4.0]],
            "g0": [6.0, 0.0],
            "CE": [[1.0], [1.0]],
            "ce0": [-3.0],
            "CI": [[1.0, 0.0, 1.0], [0.0, 1.0, 1.0]],
            "ci0": [0.0, 0.0, -2.0],
            "expect_f_hex": (12.0).hex(),
            "expect_x_hex": [(1.0).hex(), float.fromhex("0x1.0000000000002p+1").hex()],
            "expect_G_after_hex": [[(2.0).hex(), (-1.0).hex()], [(-1.0).hex(), math.sqrt(3.0).hex()]],
        }
    ],
}

if __name__ == "__main__":
    with open(os.path.join(HERE, "reference_kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1)
    print("wrote reference_kat.json")
