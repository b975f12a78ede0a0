"""Binary SoA pod traces at scale.

A pod trace of tens of millions of Alibaba instances is too large to go through per-event Python
objects and the ``k10s_scenario 1`` text.  This module streams the Alibaba v2017 CSVs straight into
the engine's binary create_pod block (``K10SPOD1``, ``include/k10s.h`` /
``scenario.pods_blob``), column by column, and decodes such a block back into numpy columns.

Semantics follow ``AlibabaWorkloadTraceV2017`` in the reference:
  * row filtering, pod naming ``{job}_{task}_{pod_no}``, cpu ``santicores * 10`` truncated to u32,
    ram ``normalized * 128 GiB`` as a saturating ``f64 as u64``, duration ``end - start``
    (src/trace/alibaba_cluster_trace_v2017/workload.rs:56-120);
  * the events are stable-sorted by start timestamp (workload.rs:140), so the block is sorted;
  * duplicated task ids are an error (workload.rs:160-161).
The result is byte-identical to ``scenario.pods_blob`` over the stable-sorted events of
``scenario.alibaba_workload_trace_from_csv`` (tests/test_trace_soa.py).

The cluster side (server_event.csv, ``AlibabaClusterTraceV2017``, cluster.rs:54-101) streams into
the ``K10SNOD1`` block the same way: ``alibaba_node_{machine_id}``, cpus x 1000 as u32, memory
x 2^37 as a saturating u64, a soft/hard error removes a node once and only one that was added,
stable-sorted by timestamp; byte-identical to ``scenario.nodes_blob`` over
``scenario.alibaba_cluster_trace_from_csv``.  A blob for k10s_engine_create_bulk is the
concatenation of such blocks (``split_blocks`` takes one apart).
"""
from __future__ import annotations

import csv
import io
from array import array
from typing import Dict, Iterable, Optional, Tuple, Union

import numpy as np

from .scenario import CPU_BASE, DENORMALIZATION_BASE, U32_MAX, _check_name, _f64_as_u64, _opt_float, _opt_int

MAGIC = b"K10SPOD1"
NODES_MAGIC = b"K10SNOD1"
# bytes a block name may not contain (k10s_builder.cpp K10S_BLOB_NAME_FORBIDDEN)
BLOB_NAME_FORBIDDEN = frozenset(b" \t\n\v\f\r#=")
_HEADER = 16


def _tasks_from_rows(rows: Iterable[list]) -> Dict[int, Tuple[Optional[int], Optional[float]]]:
    """read_batch_trace_from_str (workload.rs:150-166): task_id -> (cpus, normalized memory)."""
    tasks = {}
    for row in rows:
        if not row:
            continue
        tid = int(row[3])
        if tid in tasks:
            raise ValueError(f"duplicated task id: {tid}")
        tasks[tid] = (_opt_int(row[6]), _opt_float(row[7]))
    return tasks


def _open_text(src: Union[str, io.TextIOBase]):
    return open(src, newline="") if isinstance(src, str) else src


def alibaba_pods_blob(instances: Union[str, io.TextIOBase], tasks: Union[str, io.TextIOBase]) -> bytes:
    """Stream batch_instance.csv (path or text stream) into a sorted K10SPOD1 block.

    Only the task table is held as a dict; instance rows are reduced to four packed columns and the
    name bytes as they are read (~32 B + name length per pod); packing adds the sorted output
    (the same size again, written once) and O(n) index words (_pack_sorted)."""
    tf = _open_text(tasks)
    try:
        task_map = _tasks_from_rows(csv.reader(tf))
    finally:
        if tf is not tasks:
            tf.close()
    ts, cpu, ram, dur = array("d"), array("I"), array("Q"), array("d")
    name_len = array("I")
    names = bytearray()
    pod_no = 0
    f = _open_text(instances)
    try:
        for row in csv.reader(f):
            if not row:
                continue
            start, end, job, task = _opt_int(row[0]), _opt_int(row[1]), _opt_int(row[2]), _opt_int(row[3])
            if start is None or end is None or task is None or task not in task_map:
                continue
            cpu_sc, mem = task_map[task]
            if cpu_sc is None or mem is None:
                continue
            if start <= 0 or end <= 0 or start >= end:
                continue
            if job is None:   # workload.rs:91 unwraps job_id
                raise ValueError(f"instance of task {task} has no job id")
            name = _check_name(f"{job}_{task}_{pod_no}").encode()
            pod_no += 1
            ts.append(float(start))
            cpu.append((cpu_sc * 10) & U32_MAX)
            ram.append(_f64_as_u64(mem * float(DENORMALIZATION_BASE)))
            dur.append(float(end - start))
            name_len.append(len(name))
            names += name
    finally:
        if f is not instances:
            f.close()
    return _pack_sorted(np.frombuffer(ts, "<f8"), np.frombuffer(cpu, "<u4"), np.frombuffer(ram, "<u8"),
                        np.frombuffer(dur, "<f8"), np.frombuffer(name_len, "<u4"), names)


def _pack_sorted(ts, cpu, ram, dur, name_len, names) -> bytes:
    """The sorted K10SPOD1 block, written into one preallocated buffer.  The name bytes are gathered
    in sorted order in bounded chunks of pods, so the extra memory is O(n) words for the columns
    plus one chunk's byte indices, not several int64 arrays per name byte."""
    n = ts.size
    nbytes = len(names)
    if nbytes > U32_MAX:
        raise ValueError("pod names exceed the 4 GiB offset range of a K10SPOD1 block")
    order = np.argsort(ts, kind="stable")                       # workload.rs:140 (stable sort_by)
    lens = name_len[order].astype(np.int64)
    off = np.zeros(n + 1, dtype="<u4")
    off[1:] = np.cumsum(lens)
    pad = 4 * (n & 1)
    p_ts = _HEADER
    p_cpu = p_ts + 8 * n
    p_ram = p_cpu + 4 * n + pad
    p_dur = p_ram + 8 * n
    p_off = p_dur + 8 * n
    p_chr = p_off + 4 * (n + 1)
    out = bytearray(p_chr + nbytes)
    out[:8] = MAGIC
    out[8:16] = np.array([n], dtype="<u8").tobytes()
    for p, col, dt in ((p_ts, ts, "<f8"), (p_cpu, cpu, "<u4"), (p_ram, ram, "<u8"), (p_dur, dur, "<f8")):
        np.frombuffer(out, dt, n, p)[:] = col[order]
    np.frombuffer(out, "<u4", n + 1, p_off)[:] = off
    if n:
        src = np.frombuffer(names, np.uint8)
        src_off = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(name_len, out=src_off[1:], dtype=np.int64)
        dst = np.frombuffer(out, np.uint8, nbytes, p_chr)
        CH = 1 << 16
        for a in range(0, n, CH):                               # bounded per-chunk byte gather
            o = order[a:a + CH]
            ln = lens[a:a + CH]
            base = int(off[a])
            tot = int(off[min(a + CH, n)]) - base
            starts = np.repeat(src_off[o], ln)
            within = np.arange(tot, dtype=np.int64) - np.repeat(off[a:a + o.size].astype(np.int64) - base, ln)
            dst[base:base + tot] = src[starts + within]
    return bytes(out)


def read_pods_blob(blob: bytes) -> dict:
    """Decode a K10SPOD1 block into numpy columns (ts, cpu, ram, duration; NaN = long-running) and
    the list of pod names.  Raises ValueError on a malformed block, like k10s_engine_create_bulk."""
    if len(blob) < _HEADER or blob[:8] != MAGIC:
        raise ValueError("not a K10SPOD1 block")
    n = int(np.frombuffer(blob, "<u8", 1, 8)[0])
    fixed = n * (8 + 4 + 8 + 8) + 4 * (n & 1) + 4 * (n + 1)
    if len(blob) < _HEADER + fixed:
        raise ValueError("truncated K10SPOD1 block")
    p = _HEADER
    ts = np.frombuffer(blob, "<f8", n, p); p += 8 * n
    cpu = np.frombuffer(blob, "<u4", n, p); p += 4 * n + 4 * (n & 1)
    ram = np.frombuffer(blob, "<u8", n, p); p += 8 * n
    dur = np.frombuffer(blob, "<f8", n, p); p += 8 * n
    off = np.frombuffer(blob, "<u4", n + 1, p); p += 4 * (n + 1)
    if off[0] != 0 or np.any(np.diff(off.astype(np.int64)) < 0) or p + int(off[-1]) != len(blob):
        raise ValueError("bad name offsets in K10SPOD1 block")
    raw = blob[p:]
    names = []
    for i in range(n):   # the rules of k10s_builder.cpp parse_bulk_pods
        b = raw[off[i]:off[i + 1]]
        if not b or any(ch in BLOB_NAME_FORBIDDEN for ch in b):
            raise ValueError(f"invalid pod name {b!r} in K10SPOD1 block")
        names.append(b.decode())
    return {"ts": ts, "cpu": cpu, "ram": ram, "duration": dur, "names": names}


def alibaba_nodes_blob(machine_events: Union[str, io.TextIOBase]) -> bytes:
    """Stream server_event.csv (path or text stream) into a sorted K10SNOD1 block (cluster.rs:54-101)."""
    ts, cpu, ram, op = array("d"), array("I"), array("Q"), array("I")
    name_len = array("I")
    names = bytearray()
    created, removed = set(), set()
    f = _open_text(machine_events)
    try:
        for row in csv.reader(f):
            if not row:
                continue
            row = row + [""] * (7 - len(row))
            t, mid, etype = int(row[0]), int(row[1]), row[2]
            if etype == "add":
                c, mem = _opt_int(row[4]), _opt_float(row[5])
                if c is None or mem is None:
                    raise ValueError("add event without cpus/memory (reference unwrap panics)")
                created.add(mid)
                ts.append(float(t))
                cpu.append((c * CPU_BASE) & U32_MAX)
                ram.append(_f64_as_u64(mem * float(DENORMALIZATION_BASE)))
                op.append(0)
            elif etype in ("softerror", "harderror"):
                if mid in removed or mid not in created:
                    continue
                removed.add(mid)
                ts.append(float(t))
                cpu.append(0)
                ram.append(0)
                op.append(1)
            else:
                raise ValueError(f"Unsupported operation for a node in alibaba cluster trace: {etype}")
            name = f"alibaba_node_{mid}".encode()
            name_len.append(len(name))
            names += name
    finally:
        if f is not machine_events:
            f.close()
    n = len(ts)
    ts_a = np.frombuffer(ts, "<f8")
    order = np.argsort(ts_a, kind="stable")                     # cluster.rs:99 (stable sort_by)
    lens = np.frombuffer(name_len, "<u4")[order].astype(np.int64)
    src_off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.frombuffer(name_len, "<u4"), out=src_off[1:], dtype=np.int64)
    off = np.zeros(n + 1, dtype="<u4")
    off[1:] = np.cumsum(lens)
    src = np.frombuffer(names, np.uint8)
    out_names = bytearray(int(off[-1]))
    dst = np.frombuffer(out_names, np.uint8)
    for k, i in enumerate(order):
        dst[int(off[k]):int(off[k + 1])] = src[src_off[i]:src_off[i + 1]]
    pad = b"\0" * (4 * (n & 1))
    return (NODES_MAGIC + np.array([n], dtype="<u8").tobytes() + ts_a[order].tobytes() +
            np.frombuffer(cpu, "<u4")[order].tobytes() + pad + np.frombuffer(ram, "<u8")[order].tobytes() +
            np.frombuffer(op, "<u4")[order].tobytes() + pad + off.tobytes() + bytes(out_names))


def _block_len(blob: bytes, at: int) -> int:
    if len(blob) - at < _HEADER or blob[at:at + 8] not in (MAGIC, NODES_MAGIC):
        raise ValueError("not a K10SPOD1 / K10SNOD1 block")
    n = int(np.frombuffer(blob, "<u8", 1, at + 8)[0])
    pad = 4 * (n & 1)
    fixed = n * (8 + 4 + 8) + pad + (8 * n if blob[at:at + 8] == MAGIC else 4 * n + pad) + 4 * (n + 1)
    if len(blob) - at < _HEADER + fixed:
        raise ValueError("truncated block")
    off_end = int(np.frombuffer(blob, "<u4", 1, at + _HEADER + fixed - 4)[0])
    return _HEADER + fixed + off_end


def split_blocks(blob: bytes) -> list:
    """The blocks of a k10s_engine_create_bulk blob, in order (ValueError when malformed)."""
    out, at = [], 0
    while at < len(blob):
        ln = _block_len(blob, at)
        if at + ln > len(blob):
            raise ValueError("truncated block")
        out.append(blob[at:at + ln])
        at += ln
    return out


def read_nodes_blob(blob: bytes) -> dict:
    """Decode a K10SNOD1 block: ts, cpu, ram, op (0 create_node, 1 remove_node) columns and names,
    with the rules of k10s_builder.cpp (ValueError when malformed)."""
    if len(blob) < _HEADER or blob[:8] != NODES_MAGIC:
        raise ValueError("not a K10SNOD1 block")
    n = int(np.frombuffer(blob, "<u8", 1, 8)[0])
    pad = 4 * (n & 1)
    p = _HEADER
    if len(blob) < p + n * 24 + 2 * pad + 4 * (n + 1):
        raise ValueError("truncated K10SNOD1 block")
    ts = np.frombuffer(blob, "<f8", n, p); p += 8 * n
    cpu = np.frombuffer(blob, "<u4", n, p); p += 4 * n + pad
    ram = np.frombuffer(blob, "<u8", n, p); p += 8 * n
    op = np.frombuffer(blob, "<u4", n, p); p += 4 * n + pad
    off = np.frombuffer(blob, "<u4", n + 1, p); p += 4 * (n + 1)
    if off[0] != 0 or np.any(np.diff(off.astype(np.int64)) < 0) or p + int(off[-1]) != len(blob):
        raise ValueError("bad name offsets in K10SNOD1 block")
    if np.any(op > 1):
        raise ValueError("bad cluster op in K10SNOD1 block")
    raw = blob[p:]
    names = []
    for i in range(n):
        b = raw[off[i]:off[i + 1]]
        if not b or any(ch in BLOB_NAME_FORBIDDEN for ch in b):
            raise ValueError(f"invalid node name {b!r} in K10SNOD1 block")
        names.append(b.decode())
    return {"ts": ts, "cpu": cpu, "ram": ram, "op": op, "names": names}


def write_pods_blob(path: str, blob: bytes) -> None:
    with open(path, "wb") as f:
        f.write(blob)


def load_pods_blob(path: str) -> bytes:
    with open(path, "rb") as f:
        blob = f.read()
    read_pods_blob(blob)   # validate
    return blob


def _splitmix64(x: np.ndarray) -> np.ndarray:
    """workloads.splitmix64 over a uint64 column (wrapping arithmetic)."""
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def perturb_pods_blob(blob: bytes, seed: int, key_offset: int = 0) -> bytes:
    """Column-wise restatement of the engine's per-replica perturb_pod (k10s_engine.h,
    workloads.perturb_pod) over a K10SPOD1 block: pod k gets key ``key_offset + k`` (its position in
    the replica's workload events).  Materialises one replica's perturbed trace as a block."""
    d = read_pods_blob(blob)
    n = d["ts"].size
    key = np.arange(n, dtype=np.uint64) + np.uint64(key_offset)
    u = _splitmix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (np.uint64(0xD1B54A32D192ED03) * (key + np.uint64(1))))
    kd = (np.uint64(8) + u % np.uint64(17)).astype(np.float64)
    kc = np.uint64(12) + (u >> np.uint64(20)) % np.uint64(9)
    kr = np.uint64(12) + (u >> np.uint64(40)) % np.uint64(9)
    dur = (d["duration"] * kd) * 0.0625                          # NaN (long-running) stays NaN
    cpu = ((d["cpu"].astype(np.uint64) * kc) >> np.uint64(4)).astype("<u4")
    ram = ((d["ram"] >> np.uint64(4)) * kr).astype("<u8")
    p_cpu = _HEADER + 8 * n
    p_ram = p_cpu + 4 * n + 4 * (n & 1)
    p_dur = p_ram + 8 * n
    out = bytearray(blob)
    out[p_cpu:p_cpu + 4 * n] = cpu.tobytes()
    out[p_ram:p_ram + 8 * n] = ram.tobytes()
    out[p_dur:p_dur + 8 * n] = dur.astype("<f8").tobytes()
    return bytes(out)
