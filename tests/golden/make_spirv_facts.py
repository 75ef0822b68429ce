#!/usr/bin/env python3
"""Extract constants, names and call order from the reference's executed SPIR-V.

Reads /root/reference/shaders_spv/compute_with_dynamic_light_source.spv as
DATA (a word stream) — nothing is executed.  Writes spirv_facts.json next to
this script: the float / integer constants the shader uses, the debug names
of its functions, and the sequence of OpFunctionCall targets inside each
function.  tests/test_oracle_kat.py checks the oracle's constants and call
order against it.  Run once with the reference present; the JSON is committed.
"""
import hashlib
import json
import os
import struct
import sys

SPV = "/root/reference/shaders_spv/compute_with_dynamic_light_source.spv"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "spirv_facts.json")

OP_NAME, OP_TYPE_INT, OP_TYPE_FLOAT, OP_CONSTANT, OP_FUNCTION, OP_FUNCTION_END, OP_FUNCTION_CALL = 5, 21, 22, 43, 54, 56, 57
OP_EXT_INST = 12
OP_DECORATE, OP_MEMBER_DECORATE, DEC_NO_CONTRACTION = 71, 72, 42
OP_FADD, OP_FSUB, OP_FMUL, OP_FDIV = 129, 131, 133, 136


def main(path=SPV):
    data = open(path, "rb").read()
    words = struct.unpack("<%dI" % (len(data) // 4), data)
    assert words[0] == 0x07230203, "not SPIR-V"
    names, types, consts = {}, {}, []
    calls, cur = {}, None
    ext = []
    no_contraction = 0
    float_ops = {"OpFAdd": 0, "OpFSub": 0, "OpFMul": 0, "OpFDiv": 0}
    op_names = {OP_FADD: "OpFAdd", OP_FSUB: "OpFSub", OP_FMUL: "OpFMul", OP_FDIV: "OpFDiv"}
    i = 5
    while i < len(words):
        wc, op = words[i] >> 16, words[i] & 0xFFFF
        ins = words[i:i + wc]
        if op == OP_NAME:
            raw = struct.pack("<%dI" % (wc - 2), *ins[2:])
            names[ins[1]] = raw.split(b"\0", 1)[0].decode()
        elif op == OP_TYPE_INT:
            types[ins[1]] = ("int" if ins[3] else "uint", ins[2])
        elif op == OP_TYPE_FLOAT:
            types[ins[1]] = ("float", ins[2])
        elif op == OP_CONSTANT:
            kind, width = types.get(ins[1], ("?", 32))
            w = ins[3]
            if kind == "float":
                v = struct.unpack("<f", struct.pack("<I", w))[0]
                consts.append({"type": "float", "bits": "%08x" % w, "value": v})
            elif kind == "int":
                consts.append({"type": "int", "value": struct.unpack("<i", struct.pack("<I", w))[0]})
            else:
                consts.append({"type": "uint", "value": w})
        elif op == OP_FUNCTION:
            cur = names.get(ins[2], str(ins[2])).split("(")[0]
            calls[cur] = []
        elif op == OP_FUNCTION_END:
            cur = None
        elif op == OP_FUNCTION_CALL and cur is not None:
            calls[cur].append(names.get(ins[3], str(ins[3])).split("(")[0])
        elif op == OP_DECORATE and wc >= 3 and ins[2] == DEC_NO_CONTRACTION:
            no_contraction += 1
        elif op == OP_MEMBER_DECORATE and wc >= 4 and ins[3] == DEC_NO_CONTRACTION:
            no_contraction += 1
        elif op in op_names and cur is not None:
            float_ops[op_names[op]] += 1
        elif op == OP_EXT_INST and cur is not None:
            ext.append({"function": cur, "glsl_std_450": ins[4]})
        i += wc
    facts = {
        "source": os.path.basename(path),
        "sha256": hashlib.sha256(data).hexdigest(),
        "functions": sorted({n.split("(")[0] for n in names.values() if "(" in n}),
        "constants": consts,
        "calls": calls,
        "glsl_std_450_ops": ext,
        # GLSL `precise` becomes NoContraction; none means a driver may fuse
        # every multiply-add into an FMA (tests/golden/make_envelope.py)
        "no_contraction_decorations": no_contraction,
        "float_arith_ops": float_ops,
    }
    json.dump(facts, open(OUT, "w"), indent=1)
    print(f"wrote {OUT}: {len(consts)} constants, {len(calls)} functions")


if __name__ == "__main__":
    main(*sys.argv[1:])
