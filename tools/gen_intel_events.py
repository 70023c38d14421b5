#!/usr/bin/env python3
"""Generates src/pmu/IntelNamedEvents.inc: the named core-PMU events of every
Intel family the reference ships tables for, as one compact line each
(name -> perf "event=..,umask=..[,cmask=..][,inv=1][,edge=1][,any=1]"
[,offcore_rsp=..|,ldlat=..]), and src/pmu/IntelUncoreEvents.inc: the named
uncore events of its 16 uncore tables (CHA / CBox, IMC, M2M, M3UPI, UPI /
QPI, IIO, IRP, PCU, UBox, ...), one line each (PMU prefix, name, perf fields).

The encodings are Intel's public perfmon data, which the reference carries as
generated C++ (/root/reference/hbt/src/perf_event/json_events/generated/intel/
*_core_*.cpp, dispatched by JsonEvents.h:135+).  This script reads those files
offline (regular expressions over their EventDef initialisers), keeps the
core events only (uncore PMUs need their own sysfs types, which the runtime
JSON loader src/pmu/JsonEvents.cpp handles from perf's pmu-events JSON), and
writes the table the daemon compiles in.  Run it again only to change the
selection:

    python3 tools/gen_intel_events.py /root/reference/hbt/src/perf_event/json_events/generated/intel \\
        src/pmu/IntelNamedEvents.inc src/pmu/IntelUncoreEvents.inc
"""
import os
import re
import sys

# reference table stem -> our family key (src/pmu/IntelEvents.cpp maps CpuArch to it)
FAMILIES = {
    "skylakex_core": "skx",
    "cascadelakex_core": "clx",
    "icelake_core": "icl",
    "skylake_core": "skl",
    "broadwellx_core": "bdx",
    "broadwell_core": "bdw",
    "broadwellde_core": "bdwde",
    "haswellx_core": "hsx",
    "ivybridge_core": "ivb",
    "sandybridge_core": "snb",
    "nehalemex_core": "nhm",
    "goldmont_core": "glm",
    "snowridgex_core": "snr",
    "knightslanding_core": "knl",
}

# reference uncore table stem -> family key (experimental tables merge into theirs)
UNCORE_FAMILIES = {
    "skylakex_uncore": "skx",
    "skylakex_uncore_experimental": "skx",
    "cascadelakex_uncore": "clx",
    "cascadelakex_uncore_experimental": "clx",
    "icelake_uncore": "icl",
    "skylake_uncore": "skl",
    "broadwellx_uncore": "bdx",
    "broadwell_uncore": "bdw",
    "broadwellde_uncore": "bdwde",
    "haswellx_uncore": "hsx",
    "ivybridge_uncore": "ivb",
    "sandybridge_uncore": "snb",
    "snowridgex_uncore": "snr",
    "knightslanding_uncore": "knl",
}

EVENT_RE = re.compile(
    r'addEvent\(std::make_shared<EventDef>\(\s*PmuType::(\w+),\s*"([^"]+)",\s*EventDef::Encoding\{(.*?)\},\s*R"\((.*?)\)"',
    re.S)
FIELD_RE = re.compile(r"\.(\w+)\s*=\s*([^,}]+)")


def encoding(body: str):
    msr = re.search(r"\.msr_values\s*=\s*\{([^}]*)\}", body)
    f = {k: v.strip() for k, v in FIELD_RE.findall(re.sub(r"\.msr_values\s*=\s*\{[^}]*\}", "", body))}
    parts = []
    code = int(f.get("code", "0"), 0)
    umask = int(f.get("umask", "0"), 0)
    parts.append(f"event=0x{code:02x}")
    parts.append(f"umask=0x{umask:02x}")
    cmask = int(f.get("cmask", "0"), 0)
    if cmask:
        parts.append(f"cmask=0x{cmask:x}")
    for flag in ("inv", "edge", "any"):
        if f.get(flag) == "true":
            parts.append(f"{flag}=1")
    if msr:
        vals = [int(v, 0) for v in msr.group(1).split(",") if v.strip()]
        if vals and vals[0]:
            if code in (0xb7, 0xbb):    # OFFCORE_RESPONSE_0/1: the response MSR (perf's offcore_rsp, config1)
                parts.append(f"offcore_rsp=0x{vals[0]:x}")
            elif code == 0xcd:          # MEM_TRANS_RETIRED.LOAD_LATENCY: the latency threshold (perf's ldlat)
                parts.append(f"ldlat={vals[0]}")
            else:
                return None, code       # an MSR this table cannot express
    return ",".join(parts), code


def uncore_encoding(body: str):
    """perf fields of an uncore event, or None when it needs a filter MSR
    (CHA / CBox filters, PCU band thresholds) this table cannot express."""
    msr = re.search(r"\.msr_values\s*=\s*\{([^}]*)\}", body)
    if msr and any(int(v, 0) for v in msr.group(1).split(",") if v.strip()):
        return None
    f = {k: v.strip() for k, v in FIELD_RE.findall(re.sub(r"\.msr_values\s*=\s*\{[^}]*\}", "", body))}
    code = int(f.get("code", "0"), 0)
    umask = int(f.get("umask", "0"), 0)
    parts = [f"event=0x{code:02x}"]
    if umask:
        parts.append(f"umask=0x{umask:02x}")
    cmask = int(f.get("cmask", "0"), 0)
    if cmask:
        parts.append(f"thresh=0x{cmask:x}")  # the uncore PMUs' threshold field
    for flag in ("inv", "edge"):
        if f.get(flag) == "true":
            parts.append(f"{flag}=1")
    return ",".join(parts)


def write_uncore(src_dir: str, out_path: str) -> int:
    tables = {}
    for fn in sorted(os.listdir(src_dir)):
        stem = re.sub(r"_v[\d_]+(_experimental)?\.cpp$", lambda m: m.group(1) or "", fn)
        if stem not in UNCORE_FAMILIES or not fn.endswith(".cpp"):
            continue
        with open(os.path.join(src_dir, fn)) as f:
            text = f.read()
        fam = UNCORE_FAMILIES[stem]
        files, rows, seen, skipped = tables.setdefault(fam, ([], [], set(), [0]))
        files.append(fn)
        for pmu, name, body, brief in EVENT_RE.findall(text):
            if not pmu.startswith("uncore_"):
                continue
            enc = uncore_encoding(body)
            if enc is None:
                skipped[0] += 1
                continue
            key = (pmu, name.lower())
            if key in seen:
                continue
            seen.add(key)
            rows.append((pmu, name.lower(), enc))
    with open(out_path, "w") as out:
        out.write("// Generated by tools/gen_intel_events.py from Intel's public perfmon uncore\n"
                  "// event encodings (as carried by the reference's generated tables,\n"
                  "// /root/reference/hbt/src/perf_event/json_events/generated/intel/*_uncore_*.cpp).\n"
                  "// {PMU prefix (sysfs uncore_<box>[_<n>]), event name, perf fields}; events that\n"
                  "// need a filter MSR are left out.  Do not edit: re-run the generator.\n")
        for fam, (files, rows, _, skipped) in sorted(tables.items()):
            out.write(f"\n// {', '.join(files)}: {len(rows)} uncore events ({skipped[0]} need a filter MSR)\n")
            out.write(f"static const IntelUncoreEvent kIntelUncore_{fam}[] = {{\n")
            for pmu, name, enc in rows:
                out.write(f'    {{"{pmu}", "{name}", "{enc}"}},\n')
            out.write("};\n")
        out.write("\nstatic const IntelUncoreTable kIntelUncoreTables[] = {\n")
        for fam in sorted(tables):
            out.write(f'    {{"{fam}", kIntelUncore_{fam}, sizeof(kIntelUncore_{fam}) / sizeof(kIntelUncore_{fam}[0])}},\n')
        out.write("};\n")
    n = sum(len(t[1]) for t in tables.values())
    print(f"{out_path}: {n} uncore events in {len(tables)} families")
    return 0


def main(src_dir: str, out_path: str, uncore_path: str = "") -> int:
    tables = {}
    for fn in sorted(os.listdir(src_dir)):
        stem = re.sub(r"_v[\d_]+\.cpp$", "", fn)
        if stem not in FAMILIES or not fn.endswith(".cpp"):
            continue
        with open(os.path.join(src_dir, fn)) as f:
            text = f.read()
        rows, seen = [], set()
        for pmu, name, body, brief in EVENT_RE.findall(text):
            if pmu != "cpu":
                continue
            enc, code = encoding(body)
            if code == 0 or enc is None:  # fixed-counter pseudo events (INST_RETIRED.ANY, ...) / other MSRs
                continue
            key = name.lower()
            if key in seen:
                continue
            seen.add(key)
            rows.append((key, enc))
        tables[FAMILIES[stem]] = (fn, rows)
    with open(out_path, "w") as out:
        out.write("// Generated by tools/gen_intel_events.py from Intel's public perfmon event\n"
                  "// encodings (as carried by the reference's generated tables,\n"
                  "// /root/reference/hbt/src/perf_event/json_events/generated/intel/*_core_*.cpp).\n"
                  "// Core PMU events only.  Do not edit: re-run the generator.\n")
        for fam, (fn, rows) in sorted(tables.items()):
            out.write(f"\n// {fn}: {len(rows)} programmable core events\n")
            out.write(f"static const IntelNamedEvent kIntel_{fam}[] = {{\n")
            for name, enc in rows:
                out.write(f'    {{"{name}", "{enc}"}},\n')
            out.write("};\n")
        out.write("\nstatic const IntelNamedTable kIntelNamedTables[] = {\n")
        for fam, (fn, rows) in sorted(tables.items()):
            out.write(f'    {{"{fam}", kIntel_{fam}, sizeof(kIntel_{fam}) / sizeof(kIntel_{fam}[0])}},\n')
        out.write("};\n")
    print(f"{out_path}: {sum(len(r) for _, r in tables.values())} events in {len(tables)} families")
    if uncore_path:
        write_uncore(src_dir, uncore_path)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""))
