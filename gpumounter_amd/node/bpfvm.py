"""A tiny interpreter for the cgroup-device eBPF programs gm_host.cpp generates.

Used (1) by tests to check the *semantics* of generated allow-lists against the kernel's rules
(first match wins; requested access must be a subset of the rule's; wildcards; tail-call into the
runtime's original program), and (2) by the recording backend to audit what a recorded program
would actually allow. Supports the instruction subset the generator emits plus the common
ALU/JMP forms, a 512-byte stack, and ``bpf_map_lookup_elem`` on the allow-set HASH map of
set-mode programs (``maps``: map fd as encoded in the program → {(type, major, minor): access}).
"""
from __future__ import annotations

import struct
from typing import Callable, Dict, List, Optional, Sequence, Tuple

BPF_DEVCG_DEV_BLOCK = 1
BPF_DEVCG_DEV_CHAR = 2
ACC_MKNOD, ACC_READ, ACC_WRITE = 1, 2, 4
MASK64 = (1 << 64) - 1


class BpfError(RuntimeError):
    pass


def decode(insn: int):
    raw = struct.pack("<Q", insn)
    code, regs, off, imm = struct.unpack("<BBhi", raw)
    return code, regs & 0xF, regs >> 4, off, imm


CTX, STACK_TOP, VALUE, MAP = 0x1000, 0x10200, 0x20000, 0x40000000
_WIDTH = {0x00: 4, 0x08: 2, 0x10: 1, 0x18: 8}


def run(prog: Sequence[int], dev_type: int, access: int, major: int, minor: int,
        chained: Optional[Callable[[int, int, int, int], int]] = None, max_steps: int = 10000,
        maps: Optional[Dict[int, Dict[Tuple[int, int, int], int]]] = None) -> int:
    """Execute ``prog`` for one device access; returns r0 (1 allow / 0 deny)."""
    mem = {CTX: bytearray(struct.pack("<III", (access << 16) | dev_type, major, minor)),
           STACK_TOP - 512: bytearray(512), VALUE: bytearray(4)}

    def region(addr: int, width: int):
        for base, buf in mem.items():
            if base <= addr and addr + width <= base + len(buf):
                return buf, addr - base
        raise BpfError(f"memory access out of bounds at {addr:#x}")

    regs = [0] * 11
    regs[1] = CTX
    regs[10] = STACK_TOP
    pc = 0
    steps = 0
    while True:
        steps += 1
        if steps > max_steps or pc < 0 or pc >= len(prog):
            raise BpfError(f"pc out of range or runaway at {pc}")
        code, dst, src, off, imm = decode(prog[pc])
        cls = code & 0x07
        if code == 0x18:  # ld_imm64 (map fd pseudo or constant)
            _, _, _, _, imm2 = decode(prog[pc + 1])
            if src == 1:   # BPF_PSEUDO_MAP_FD
                regs[dst] = MAP + (imm & 0xFFFF)
            else:
                regs[dst] = ((imm2 & 0xFFFFFFFF) << 32) | (imm & 0xFFFFFFFF)
            pc += 2
            continue
        if cls == 0x01:  # LDX
            width = _WIDTH[code & 0x18]
            buf, o = region(regs[src] + off, width)
            regs[dst] = int.from_bytes(buf[o:o + width], "little")
            pc += 1
            continue
        if cls == 0x03:  # STX
            width = _WIDTH[code & 0x18]
            buf, o = region(regs[dst] + off, width)
            buf[o:o + width] = (regs[src] & ((1 << (8 * width)) - 1)).to_bytes(width, "little")
            pc += 1
            continue
        if cls in (0x07, 0x04):  # ALU64 / ALU
            op = code & 0xF0
            val = regs[src] if code & 0x08 else imm & MASK64
            a = regs[dst]
            if op == 0xB0:
                r = val
            elif op == 0x50:
                r = a & val
            elif op == 0x40:
                r = a | val
            elif op == 0x00:
                r = a + val
            elif op == 0x10:
                r = a - val
            elif op == 0x70:
                r = a >> (val & 63)
            elif op == 0x60:
                r = a << (val & 63)
            elif op == 0xA0:
                r = a ^ val
            else:
                raise BpfError(f"unsupported alu op {code:#x}")
            r &= MASK64
            if cls == 0x04:
                r &= 0xFFFFFFFF
            regs[dst] = r
            pc += 1
            continue
        if cls == 0x05:  # JMP
            op = code & 0xF0
            if op == 0x90:  # exit
                return regs[0]
            if op == 0xF0:  # BPF_TAIL_CALL: the verifier's rewrite of bpf_tail_call (xlated)
                if chained is None:
                    pc += 1
                    continue
                return chained(dev_type, access, major, minor)
            if op == 0x80 and imm == 1:  # bpf_map_lookup_elem(map, key)
                table = (maps or {}).get(regs[1] - MAP)
                if table is None:
                    raise BpfError(f"lookup in unknown map {regs[1] - MAP}")
                buf, o = region(regs[2], 12)
                key = struct.unpack("<III", bytes(buf[o:o + 12]))
                val = table.get(key)
                if val is None:
                    regs[0] = 0
                else:
                    mem[VALUE][:] = struct.pack("<I", val & 0xFFFFFFFF)
                    regs[0] = VALUE
                regs[1:6] = [0] * 5   # caller-saved registers are clobbered
                pc += 1
                continue
            if op == 0x80:  # call
                if imm != 12:
                    raise BpfError(f"unsupported helper {imm}")
                if chained is None:
                    pc += 1  # tail call into an empty slot falls through
                    continue
                return chained(dev_type, access, major, minor)
            val = regs[src] if code & 0x08 else imm & MASK64
            a = regs[dst]
            take = {0x00: True, 0x10: a == val, 0x50: a != val, 0x20: a > val, 0x30: a >= val,
                    0xA0: a < val, 0xB0: a <= val, 0x40: bool(a & val)}.get(op)
            if take is None:
                raise BpfError(f"unsupported jmp {code:#x}")
            pc += 1 + (off if take else 0)
            continue
        raise BpfError(f"unsupported opcode {code:#x}")


def runtime_default(dev_type: int, access: int, major: int, minor: int) -> int:
    """runc's default device policy (what a freshly started container allows)."""
    if access == ACC_MKNOD:
        return 1
    if dev_type != BPF_DEVCG_DEV_CHAR:
        return 0
    allowed = {(1, 3), (1, 5), (1, 7), (1, 8), (1, 9), (5, 0), (5, 1), (5, 2), (10, 200)}
    return 1 if (major, minor) in allowed or major == 136 else 0


def immediates(prog: Sequence[int]) -> set:
    """Constants the program compares against (jump-with-immediate operands): for a generated
    allow-list these are exactly the rule majors/minors, i.e. the only interesting inputs."""
    out = set()
    skip = False
    for insn in prog:
        if skip:
            skip = False
            continue
        code, _, _, _, imm = decode(insn)
        if code == 0x18:
            skip = True
            continue
        if code & 0x07 in (0x05, 0x06) and not code & 0x08 and code & 0xF0 not in (
                0x00, 0x80, 0x90, 0xF0):
            out.add(imm & 0xFFFFFFFF)
    return out


def allowed_pairs(prog: List[int], candidates, chained=runtime_default, maps=None):
    """(major, minor) pairs from ``candidates`` the program allows for rw char access."""
    out = set()
    for ma, mi in candidates:
        if run(prog, BPF_DEVCG_DEV_CHAR, ACC_READ | ACC_WRITE, ma, mi, chained, maps=maps):
            out.add((ma, mi))
    return out
