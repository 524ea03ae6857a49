#!/usr/bin/env python3
"""Record the reference's SFMT19937 known answers as a fixture.

src/tests/test_random.cpp:434-507 (TestRandom::test00_validate) lists the first
198 outputs of Random(4321)->nextULong() for Mitsuba's SFMT19937.  This script
copies those numbers (data, not code) into tests/golden/sfmt_4321.json.  Run it
where /root/reference exists; the fixture is committed and travels.
"""
import json
import os
import re
import sys

SRC = "/root/reference/src/tests/test_random.cpp"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    if not os.path.exists(SRC):
        print("no reference here; the fixture is already committed")
        return 0
    text = open(SRC).read()
    body = text[text.index("void TestRandom::test00_validate()"):]
    body = body[:body.index("};")]
    values = re.findall(r"0x([0-9a-fA-F]{16})ULL", body)
    seed = int(re.search(r"new Random\((\d+)\)", text[text.index("void TestRandom::test00_validate()"):]).group(1))
    with open(os.path.join(HERE, "sfmt_4321.json"), "w") as f:
        json.dump({"source": "src/tests/test_random.cpp:434-507 (TestRandom::test00_validate)",
                   "seed": seed, "next_ulong": ["0x" + v.lower() for v in values]}, f, indent=0)
    print("%d values, seed %d" % (len(values), seed))
    return 0


if __name__ == "__main__":
    sys.exit(main())
