"""Canonical-state checksum computed from the canonical JSON (third, independent statement of
the checksum definition in DESIGN.md; checks the C++ oracle and device checksums).
TEST INFRASTRUCTURE ONLY."""

M64 = (1 << 64) - 1
MARKER_TAG = 0x4D41524B45520000


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def fnv1a(b):
    h = 0xCBF29CE484222325
    for c in b:
        h ^= c
        h = (h * 0x100000001B3) & M64
    return h


def seg_hash(idx, text_hash, seq, client, rseq, rclient, overlap, props_lo, props_defined):
    b = (seq & 0xFFFFFFFF) | ((client & 0xFFFFFFFF) << 32)
    c = (rseq & 0xFFFFFFFF) | ((rclient & 0xFFFFFFFF) << 32)
    h = mix64(text_hash ^ ((idx * 0xD6E8FEB86659FD93) & M64))
    h = mix64(h ^ b)
    h = mix64(h ^ c)
    h = mix64(h ^ overlap)
    h = mix64(h ^ props_lo ^ ((1 if props_defined else 0) << 63))
    return h


def ovl_term(mask, ovx):
    """the overlap term: ids < 64 as a bitmask, ids >= 64 hashed in (ovx_hash)"""
    return mask ^ mix64(ovx ^ 0x4F56584944530000) if ovx else mask


def ovx_hash(ids):
    """the ids >= 64, ascending: up to eight below 256 as their byte list, any other list folded id by
    id (mt_checksum.h mt_ovx_hash)"""
    if not ids:
        return 0
    if len(ids) <= 8 and max(ids) <= 255:
        return sum(o << (8 * q) for q, o in enumerate(ids))
    h = 0x9E3779B97F4A7C15
    for o in ids:
        h = mix64(h ^ o)
    return h or 1


def props_term(lo, hi, xlo, xhi, y0=0, y1=0, y2=0, y3=0):
    """the props term: low bytes of keys 0..7; high bytes and keys 8..15 hashed in, then keys 16..31
    (low / high bytes of 16..23, of 24..31) when any is set"""
    t = lo
    if hi | xlo | xhi:
        t ^= mix64(mix64(hi ^ 0x1111111111111111) ^ mix64(xlo ^ 0x2222222222222222) ^
                   mix64(xhi ^ 0x3333333333333333))
    if y0 | y1 | y2 | y3:
        t ^= mix64(mix64(y0 ^ 0x4444444444444444) ^ mix64(y1 ^ 0x5555555555555555) ^
                   mix64(y2 ^ 0x6666666666666666) ^ mix64(y3 ^ 0x7777777777777777))
    return t


def utf16_units(text):
    """a str as its UTF-16 code units (lone surrogates included, as JSON carries them)"""
    b = text.encode('utf-16-le', 'surrogatepass')
    return [b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2)]


def checksum(state):
    """state: canonical JSON dict {"seq","msn","segs":[[text,seq,client,rseq,rclient,[ov],props]],"tree"}"""
    seg_sum = 0
    for i, (text, seq, client, rseq, rclient, ov, props) in enumerate(state['segs']):
        mask = sum(1 << o for o in set(ov) if o < 64)
        ovx = ovx_hash(sorted(o for o in set(ov) if o >= 64))
        w = [0] * 8
        if props is not None:
            for k, v in props.items():
                kid, v = int(k[1:]), int(v)
                w[(kid >> 3) * 2] |= (v & 0xFF) << (8 * (kid & 7))
                w[(kid >> 3) * 2 + 1] |= (v >> 8) << (8 * (kid & 7))
        overlap, props_lo = ovl_term(mask, ovx), props_term(*w)
        if isinstance(text, dict):  # a Marker {"marker": refType}: its refType byte, tagged
            th = fnv1a(bytes([text['marker']])) ^ MARKER_TAG
        else:
            th = fnv1a(utf16_units(text))
        seg_sum = (seg_sum + seg_hash(i, th, seq, client, rseq, rclient, overlap, props_lo,
                                      props is not None)) & M64
    tree_sum = 0
    for level, counts in enumerate(state['tree']):
        for b, cnt in enumerate(counts):
            tree_sum = (tree_sum + mix64(cnt ^ (b << 8) ^ (level << 56))) & M64
    s = mix64(seg_sum) ^ mix64(tree_sum ^ 0x5851F42D4C957F2D)
    s ^= mix64((state['seq'] & 0xFFFFFFFF) | ((state['msn'] & 0xFFFFFFFF) << 32))
    return mix64(s ^ len(state['segs']))


def text_of(state):
    return ''.join(s[0] for s in state['segs'] if s[3] == -1 and not isinstance(s[0], dict))
