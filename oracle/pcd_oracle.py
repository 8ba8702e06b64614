"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of the PCD v0.7 writer/reader and the
LZF codec of the reference (pcd_helper.h:321-371 generateHeader, :489-610 writeBinary,
:628-790 writeBinaryCompressed; lzf.cpp:86-415), the checker of libpcp's pcp_pcd_* /
pcp_lzf_*.  The reference's own codec cannot be built here (lzf.cpp includes stdafx.h ->
Boost, absent), so parity is pinned by this independent line-by-line restatement and by the
LZF format's decode of its own output; the reference holds no PCD fixture."""
import numpy as np

HLOG = 13


def _slot(h):
    return ((h >> (3 * 8 - HLOG)) - h) & ((1 << HLOG) - 1)


def lzf_compress(data, out_len):
    """lzfCompress: returns the compressed bytes or None (0)."""
    ip_ = bytes(data)
    n = len(ip_)
    if n == 0 or out_len == 0:
        return None
    htab = [0] * (1 << HLOG)
    out = bytearray(out_len + 8)
    ip, op, lit = 0, 1, 0
    in_end, out_end = n, out_len

    def byte(i):
        return ip_[i] if i < n else 0  # the reference reads ip[1] of a 1-byte input (unused)
    hval = ((byte(0) << 8) | byte(1)) & 0xffffffff
    while ip < in_end - 2:
        hval = ((hval << 8) | ip_[ip + 2]) & 0xffffffff
        s = _slot(hval)
        ref = htab[s]
        htab[s] = ip
        off = ip - ref - 1
        if ref < ip and off < (1 << 13) and ref > 0 and ip_[ref + 2] == ip_[ip + 2] and \
                ip_[ref] == ip_[ip] and ip_[ref + 1] == ip_[ip + 1]:
            ln = 2
            maxlen = min(in_end - ip - ln, (1 << 8) + (1 << 3))
            if op + 3 + 1 >= out_end and op - (0 if lit else 1) + 3 + 1 >= out_end:
                return None
            out[op - lit - 1] = (lit - 1) & 0xff
            op -= 0 if lit else 1
            stop = False
            if maxlen > 16:
                for _ in range(16):
                    ln += 1
                    if ip_[ref + ln] != ip_[ip + ln]:
                        stop = True
                        break
            if not stop:
                while True:
                    ln += 1
                    if not (ln < maxlen and ip_[ref + ln] == ip_[ip + ln]):
                        break
            ln -= 2
            ip += 1
            if ln < 7:
                out[op] = ((off >> 8) + (ln << 5)) & 0xff
                op += 1
            else:
                out[op] = ((off >> 8) + (7 << 5)) & 0xff
                out[op + 1] = (ln - 7) & 0xff
                op += 2
            out[op] = off & 0xff
            op += 1
            lit = 0
            op += 1
            ip += ln + 1
            if ip >= in_end - 2:
                break
            ip -= 1
            hval = (ip_[ip] << 8) | ip_[ip + 1]
            hval = ((hval << 8) | ip_[ip + 2]) & 0xffffffff
            htab[_slot(hval)] = ip
            ip += 1
        else:
            if op >= out_end:
                return None
            lit += 1
            out[op] = ip_[ip]
            op += 1
            ip += 1
            if lit == 32:
                out[op - lit - 1] = lit - 1
                lit = 0
                op += 1
    if op + 3 > out_end:
        return None
    while ip < in_end:
        lit += 1
        out[op] = ip_[ip]
        op += 1
        ip += 1
        if lit == 32:
            out[op - lit - 1] = lit - 1
            lit = 0
            op += 1
    out[op - lit - 1] = (lit - 1) & 0xff
    op -= 0 if lit else 1
    return bytes(out[:op])


def lzf_decompress(data, out_len):
    d = bytes(data)
    out = bytearray()
    i = 0
    while i < len(d):
        ctrl = d[i]
        i += 1
        if ctrl < 32:
            out += d[i:i + ctrl + 1]
            i += ctrl + 1
        else:
            ln = ctrl >> 5
            if ln == 7:
                ln += d[i]
                i += 1
            ref = len(out) - ((ctrl & 0x1f) << 8) - 1 - d[i]
            i += 1
            for k in range(ln + 2):
                out.append(out[ref + k])
    return bytes(out) if len(out) <= out_len else None


HEADER = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgba stamp_id\nSIZE 8 8 8 4 4\n"
          "TYPE F F F U U\nCOUNT 1 1 1 1 1\nWIDTH {w}\nHEIGHT {h}\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA {d}\n")


def pcd_bytes(cloud, compressed=False, width=0, height=0):
    """The file writeBinary / writeBinaryCompressed produce for a PointXYZRGBA cloud."""
    n = len(cloud)
    w, h = (width, height) if width > 0 and height > 0 else (n, 1)
    head = HEADER.format(w=w, h=h, n=n, d="binary_compressed" if compressed else "binary").encode()
    cols = [cloud["x"].astype("<f8"), cloud["y"].astype("<f8"), cloud["z"].astype("<f8"),
            cloud["rgba"].astype("<u4"), cloud["stamp_id"].astype("<u4")]
    if not compressed:
        rec = np.zeros(n, dtype=[("x", "<f8"), ("y", "<f8"), ("z", "<f8"), ("rgba", "<u4"), ("stamp_id", "<u4")])
        for name, c in zip(rec.dtype.names, cols):
            rec[name] = c
        return head + rec.tobytes()
    planes = b"".join(c.tobytes() for c in cols)
    comp = lzf_compress(planes, int(np.float32(len(planes)) * np.float32(1.5)))
    return head + np.array([len(comp), len(planes)], dtype="<u4").tobytes() + comp
