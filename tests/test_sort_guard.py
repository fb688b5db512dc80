"""Guard for the rocPRIM finding of round 4 (tools/sort_probe, profiles/r04/sort_probe,
DESIGN.md §5): ROCm 7.2's radix_sort_keys on 64-bit keys over a bit range that
starts above bit 0 and ends at bit 64 returns a non-permutation for 3 k-1 Mi
keys.  Every device sort in the library therefore starts at bit 0; this test
fails if a rocPRIM radix sort call in csrc/ passes any other begin_bit."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "dynamicgraphrepresentationlearning_amd", "csrc")


def _calls(src: str):
    """(name, [args]) of every rocprim::*radix_sort_*( call, comments stripped."""
    src = re.sub(r"//[^\n]*", "", src)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    for m in re.finditer(r"rocprim::(\w*radix_sort\w*)\s*\(", src):
        i, depth, args, cur = m.end(), 1, [], ""
        while depth:
            c = src[i]
            if c in "([{":
                depth += 1
            elif c in ")]}":
                depth -= 1
            if depth == 1 and c == ",":
                args.append(cur.strip())
                cur = ""
            elif depth:
                cur += c
            i += 1
        args.append(cur.strip())
        yield m.group(1), args


def test_every_radix_sort_starts_at_bit_0():
    seen = 0
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith((".hip", ".h", ".cpp")):
            continue
        for name, args in _calls(open(os.path.join(CSRC, f)).read()):
            seen += 1
            # (..., begin_bit, end_bit, stream[, debug]): the stream is the last argument here
            assert len(args) >= 3, (f, name, args)
            begin = args[-3]
            assert re.fullmatch(r"0u?", begin), f"{f}: {name} begin_bit = {begin!r} (must be 0; see module doc)"
    assert seen >= 4, "no rocPRIM radix sort calls found: the guard's parser is stale"
