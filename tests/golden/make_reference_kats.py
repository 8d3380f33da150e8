"""Generate tests/golden/reference_kats.json from ringpop-go's own test assertions.

The expected values are transcribed from the reference tests' `expected :=` expressions. They
are NOT computed by the oracle, so the oracle is checked against them.
"""
import json
import os

STATUSES = [0, 1, 2, 3, 4]  # alive, suspect, faulty, leave, tombstone (member_test.go:49)


def states(inc0=1000):
    return [(inc0 + i, st) for i in range(4) for st in STATUSES]  # member_test.go:50-57


def main():
    s = states()
    # member_test.go:82-85: expected := j > i
    non_local = [[int(j > i) for j in range(20)] for i in range(20)]
    # member_test.go:107-108: (c.Status == Suspect || Faulty || Tombstone) && c.Incarnation >= m.Incarnation
    local = [[int(s[j][1] in (1, 2, 4) and s[j][0] >= s[i][0]) for j in range(20)] for i in range(20)]
    out = {
        "source": "maniacs-ops/ringpop-go swim/member_test.go:77-121",
        "states": s,
        "non_local_override_20x20": non_local,
        "local_override_20x20": local,
        "maxp_11_nodes": 30,  # node_bootstrap_test.go:196-200
        "heal_with_faulties": {  # heal_partition_test.go:61-76
            "after_first_heal": {"A_sees_A": [3, "alive"], "A_sees_B": [0, "faulty"],
                                 "B_sees_B": [5, "alive"], "B_sees_A": [0, "faulty"]},
            "after_second_heal": {"A_sees_A": [3, "alive"], "A_sees_B": [5, "alive"],
                                  "B_sees_B": [5, "alive"], "B_sees_A": [3, "alive"]},
        },
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=None, separators=(",", ":"))
        f.write("\n")


if __name__ == "__main__":
    main()
