"""Generate tests/golden/retention_cases.json from the reference's own table-driven test.

Run in the build container only (it reads /root/reference, which does not exist on the GPU box):

    python tests/golden/make_retention_cases.py          # writes the fixture
    python tests/golden/make_retention_cases.py --check  # compares with the committed fixture

Source: the #[case(RetentionIteratorTestCase { ... })] attributes of
test_retention_iterator_table_driven (slatedb/src/retention_iterator.rs:643-1023).  Data only: each
case's name, input entries, retention_timeout (seconds; null = None), retention_min_seq,
compaction_start_ts, expected entries and filter_tombstone.  system_clock_ts equals
compaction_start_ts (1000) in every case; the harness passes an empty SequenceTracker
(retention_iterator.rs:1027-1048), so a timeout > 0 keeps every seq inside the time window.

Entries are [key, kind (0 value, 1 merge, 2 tombstone), value, seq, create_ts, expire_ts] from
RowEntry::new_value / new_merge / new_tombstone and .with_create_ts / .with_expire_ts.
"""
import json
import os
import re
import sys

REF = os.environ.get("SDB_REFERENCE", "/root/reference")
SRC = os.path.join(REF, "slatedb", "src", "retention_iterator.rs")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "retention_cases.json")
SOURCE_NOTE = ("slatedb/src/retention_iterator.rs:655-1024 (test_retention_iterator_table_driven): inputs and "
               "expected entries; system_clock_ts = compaction_start_ts = 1000, empty SequenceTracker "
               "(find_ts -> None -> now), so a timeout > 0 keeps every seq in the time window and a zero / "
               "absent timeout none. Entries: [key, kind(0 value,1 merge,2 tombstone), value, seq, create_ts, "
               "expire_ts]")


def strip_comments(txt):
    return re.sub(r"//[^\n]*", "", txt)


def split_top(s, sep=","):
    """Split on `sep` at bracket depth 0 (outside string literals)."""
    out, depth, cur, i, instr = [], 0, [], 0, False
    while i < len(s):
        c = s[i]
        if instr:
            cur.append(c)
            if c == "\\":
                cur.append(s[i + 1])
                i += 2
                continue
            if c == '"':
                instr = False
        elif c == '"':
            instr = True
            cur.append(c)
        elif c in "([{":
            depth += 1
            cur.append(c)
        elif c in ")]}":
            depth -= 1
            cur.append(c)
        elif c == sep and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(c)
        i += 1
    if "".join(cur).strip():
        out.append("".join(cur).strip())
    return out


def bstr(tok):
    m = re.fullmatch(r'b"((?:[^"\\]|\\.)*)"', tok.strip())
    if not m:
        raise ValueError("not a byte string: " + tok)
    return m.group(1)


def entry(expr):
    """RowEntry::new_*(...)[.with_create_ts(x)][.with_expire_ts(y)] -> list."""
    m = re.match(r"RowEntry::(new_value|new_merge|new_tombstone)\((.*?)\)((?:\s*\.with_\w+\([^)]*\))*)\s*$",
                 expr.strip(), re.S)
    if not m:
        raise ValueError("unparsed entry: " + expr)
    ctor, args, chain = m.group(1), split_top(m.group(2)), m.group(3)
    if ctor == "new_tombstone":
        key, kind, val, seq = bstr(args[0]), 2, "", int(args[1])
    else:
        key, kind, val, seq = bstr(args[0]), 0 if ctor == "new_value" else 1, bstr(args[1]), int(args[2])
    cts = ets = None
    for name, v in re.findall(r"\.with_(\w+)\(([^)]*)\)", chain):
        if name == "create_ts":
            cts = int(v)
        elif name == "expire_ts":
            ets = int(v)
        else:
            raise ValueError("unknown builder call " + name)
    return [key, kind, val, seq, cts, ets]


def entries(vec_expr):
    m = re.fullmatch(r"vec!\[(.*)\]", vec_expr.strip(), re.S)
    return [entry(e) for e in split_top(m.group(1))] if m.group(1).strip() else []


def timeout(expr):
    e = expr.strip()
    if e == "None":
        return None
    if e == "Some(Duration::ZERO)":
        return 0
    m = re.fullmatch(r"Some\(Duration::from_secs\((\d+)\)\)", e)
    if not m:
        raise ValueError("unparsed timeout " + e)
    return int(m.group(1))


def opt_int(expr):
    e = expr.strip()
    if e == "None":
        return None
    return int(re.fullmatch(r"Some\((\d+)\)", e).group(1))


def extract():
    src = strip_comments(open(SRC, encoding="utf-8").read())
    cases = []
    for body in re.findall(r"#\[case\(RetentionIteratorTestCase \{(.*?)\}\)\]", src, re.S):
        fields = {}
        for f in split_top(body):
            k, v = f.split(":", 1)
            fields[k.strip()] = v.strip()
        sys_ts, cst = int(fields["system_clock_ts"]), int(fields["compaction_start_ts"])
        if sys_ts != cst:
            raise ValueError("system_clock_ts != compaction_start_ts in " + fields["name"])
        cases.append({"name": json.loads(fields["name"]), "input": entries(fields["input_entries"]),
                      "timeout_s": timeout(fields["retention_timeout"]),
                      "retention_min_seq": opt_int(fields["retention_min_seq"]), "compaction_start_ts": cst,
                      "expected": entries(fields["expected_entries"]),
                      "filter_tombstone": fields["filter_tombstone"] == "true"})
    return {"source": SOURCE_NOTE, "cases": cases}


def main():
    if not os.path.exists(SRC):
        sys.exit("reference not found at %s" % SRC)
    data = extract()
    if "--check" in sys.argv:
        have = json.load(open(OUT))
        if have["cases"] != data["cases"]:
            sys.exit("retention_cases.json differs from the reference table")
        print("retention_cases.json matches the reference (%d cases)" % len(data["cases"]))
        return
    json.dump(data, open(OUT, "w"), indent=1)
    print("wrote %s (%d cases)" % (OUT, len(data["cases"])))


if __name__ == "__main__":
    main()
