"""Extract the model_simple parameter set from the reference DLL's bytes -> gen/params.json.

BUILD-TIME DATA EXTRACTION (shared by the oracle and the product tables).  This script only *reads* the PE file as bytes
(`/root/reference/core/model_simple_win64.dll`); it never loads or executes it.
It walks the Simulink C-API map that the DLL embeds (rtwCAPI_ModelMappingStaticInfo at
dll.data@0x24580, returned by `model_simple_GetCAPIStaticMap` dll@0x36b0; address map at
dll.data@0x240c0) and records every block/model parameter by its Simulink path.
SURVEY.md Appendix B/C documents the same values; this makes the extraction reproducible.

Usage:  python gen/extract_params.py [path/to/model_simple_win64.dll]
"""
import json
import os
import struct
import sys

IMAGE_BASE = 0x180000000
MMI = 0x24580          # rtwCAPI_ModelMappingStaticInfo
ADDR_MAP = 0x240c0     # rtDataAddrMap (void*[])


class PE:
    def __init__(self, path):
        self.b = open(path, "rb").read()
        pe = struct.unpack_from("<I", self.b, 0x3C)[0]
        nsec = struct.unpack_from("<H", self.b, pe + 6)[0]
        optsz = struct.unpack_from("<H", self.b, pe + 20)[0]
        off = pe + 24 + optsz
        self.secs = []
        for _ in range(nsec):
            vsz, va, rsz, rptr = struct.unpack_from("<IIII", self.b, off + 8)
            self.secs.append((va, vsz, rptr, rsz))
            off += 40

    def read(self, rva, n):
        for va, vsz, rptr, rsz in self.secs:
            if va <= rva < va + max(vsz, rsz):
                o = rva - va
                raw = self.b[rptr + o: rptr + min(o + n, rsz)] if o < rsz else b""
                return raw + b"\0" * (n - len(raw))  # bytes past SizeOfRawData are .bss zeros
        raise ValueError(hex(rva))

    def u(self, rva, fmt):
        return struct.unpack(fmt, self.read(rva, struct.calcsize(fmt)))

    def ptr(self, rva):
        v = self.u(rva, "<Q")[0]
        return v - IMAGE_BASE if v else 0

    def cstr(self, rva):
        out = bytearray()
        while True:
            c = self.read(rva + len(out), 1)
            if c == b"\0":
                break
            out += c
        try:
            return out.decode("utf-8")
        except UnicodeDecodeError:
            return out.decode("cp1251")


def extract(path):
    pe = PE(path)
    bp, nbp = pe.ptr(MMI + 0x30), pe.u(MMI + 0x38, "<I")[0]
    mp, nmp = pe.ptr(MMI + 0x40), pe.u(MMI + 0x48, "<I")[0]
    dtm, dimmap, dimarr = pe.ptr(MMI + 0x60), pe.ptr(MMI + 0x68), pe.ptr(MMI + 0x88)

    def addr(i):
        return pe.ptr(ADDR_MAP + 8 * i)

    def dims(di):
        _, ai, nd = pe.u(dimmap + 16 * di, "<IIB")
        return [pe.u(dimarr + 4 * (ai + k), "<I")[0] for k in range(nd)]

    def dsize(dt):  # rtwCAPI_DataTypeMap (32 B): cName*, mwName*, numElements, elemMapIndex, dataSize
        return pe.u(dtm + 32 * dt + 20, "<H")[0]

    def values(a, d, dt):
        n = 1
        for x in d:
            n *= x
        sz = dsize(dt)
        if sz == 8:
            return list(pe.u(a, "<%dd" % n))
        if sz == 4:
            return list(pe.u(a, "<%dI" % n))
        return list(pe.u(a, "<%dB" % n))

    block, model = {}, {}
    for i in range(nbp):  # rtwCAPI_BlockParameters, 32 B
        e = bp + 32 * i
        ami = pe.u(e, "<I")[0]
        path = pe.cstr(pe.ptr(e + 8))
        name = pe.cstr(pe.ptr(e + 16))
        dt, di = pe.u(e + 24, "<HH")
        d = dims(di)
        block[path + "." + name] = {"rva": addr(ami), "dims": d, "value": values(addr(ami), d, dt)}
    for i in range(nmp):  # rtwCAPI_ModelParameters, 24 B
        e = mp + 24 * i
        ami = pe.u(e, "<I")[0]
        name = pe.cstr(pe.ptr(e + 8))
        dt, di = pe.u(e + 16, "<HH")
        d = dims(di)
        model[name] = {"rva": addr(ami), "dims": d, "value": values(addr(ami), d, dt)}
    return {"source": "core/model_simple_win64.dll (.data, via embedded Simulink C-API map)",
            "block_parameters": block, "model_parameters": model}


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/core/model_simple_win64.dll"
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "params.json")
    data = extract(src)
    with open(out, "w", encoding="utf-8") as f:
        json.dump(data, f, ensure_ascii=False, indent=1)
    print("wrote", out, len(data["block_parameters"]), "block params,", len(data["model_parameters"]), "model params")
