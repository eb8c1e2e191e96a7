"""Generate the golden BLAKE2f fixtures in tests/golden/blake2f_golden.json.

Run in the build container (python3 tests/golden/make_golden.py). The output is committed;
nothing here runs on the GPU box.

Sources of truth (none of them is this repository's code):
  * Python's hashlib.blake2b (RFC 7693). For a message of <= 128 bytes the digest equals
    F(h = IV ^ param_block, m = zero-padded block, t = [len, 0], f = 1, rounds = 12): the
    one-block cases pin the final state of a 12-round compression; two-block cases pin
    F(F(h, m1, t=128, f=0), m2, t=len, f=1), i.e. the f = 0 path through a chained call.
  * The reference's one BLAKE2f known-answer vector, blake2f-circuit/src/blake2f.rs:193-247
    (EIP-152 example: rounds 12, h = IV with h0 ^= 0x01010040, m = "abc", t = [3, 0], f = 1).
  * rounds = 0 vectors computed from the definition alone (no G calls:
    h'_i = h_i ^ v_i ^ v_{i+8} with v the initialised work vector, README.md:14-30).
  * The spread-table rows the reference's lookup test writes (spread_table.rs:684-685) and
    the tag-boundary rows it lists (spread_table.rs:717-724), plus rows from the interleave
    formula it gives (spread_table.rs:729-736).
"""
import hashlib
import json
import os
import random
import struct

IV = [0x6a09e667f3bcc908, 0xbb67ae8584caa73b, 0x3c6ef372fe94f82b, 0xa54ff53a5f1d36f1,
      0x510e527fade682d1, 0x9b05688c2b3e6c1f, 0x1f83d9abfb41bd6b, 0x5be0cd19137e2179]
M64 = (1 << 64) - 1


def words(b, n):
    return list(struct.unpack("<%dQ" % n, b))


def hexw(ws):
    return ["%016x" % w for w in ws]


def param_h(digest_size, key_len, salt=b"", person=b""):
    p = bytearray(64)
    p[0] = digest_size
    p[1] = key_len
    p[2] = 1  # fanout
    p[3] = 1  # depth
    p[32:32 + len(salt)] = salt
    p[48:48 + len(person)] = person
    pw = words(bytes(p), 8)
    return [IV[i] ^ pw[i] for i in range(8)]


def blocks_of(data):
    """BLAKE2b padding: 128-byte blocks, last one zero padded, at least one block."""
    if not data:
        return [bytes(128)]
    out = []
    for i in range(0, len(data), 128):
        blk = data[i:i + 128]
        out.append(blk + bytes(128 - len(blk)))
    return out


def hash_case(name, msg, digest_size=64, key=b"", salt=b"", person=b""):
    """Express hashlib.blake2b(...) as a chain of F calls; expected = the digest bytes."""
    h0 = param_h(digest_size, len(key), salt, person)
    data = (key + bytes(128 - len(key)) if key else b"") + msg
    blks = blocks_of(data) if data else [bytes(128)]
    total = len(data)
    chain = []
    for i, blk in enumerate(blks):
        last = i == len(blks) - 1
        t = total if last else 128 * (i + 1)
        chain.append({"m": hexw(words(blk, 16)), "t": ["%016x" % (t & M64), "%016x" % (t >> 64)],
                      "f": 1 if last else 0, "rounds": 12})
    digest = hashlib.blake2b(msg, digest_size=digest_size, key=key, salt=salt,
                             person=person).digest()
    return {"name": name, "h": hexw(h0), "chain": chain, "digest": digest.hex(),
            "digest_size": digest_size}


def rounds0(h, t, f):
    v = list(h) + list(IV)
    v[12] ^= t[0]
    v[13] ^= t[1]
    if f:
        v[14] ^= M64
    return [h[i] ^ v[i] ^ v[i + 8] for i in range(8)]


def spread16(x):
    s = 0
    for b in range(16):
        s |= ((x >> b) & 1) << (2 * b)
    return s


def interleave_u16_with_zeros(word):
    # the shift-mask form written out at spread_table.rs:729-736
    word = (word ^ (word << 8)) & 0x00ff00ff
    word = (word ^ (word << 4)) & 0x0f0f0f0f
    word = (word ^ (word << 2)) & 0x33333333
    word = (word ^ (word << 1)) & 0x55555555
    return word


def get_tag(x):
    return 0 if x < (1 << 8) else (1 if x < (1 << 15) else 2)


def main():
    rng = random.Random(0x5962be5d)
    cases = []
    for n in (0, 1, 3, 64, 111, 127, 128):
        cases.append(hash_case("unkeyed_len%d" % n, bytes(rng.getrandbits(8) for _ in range(n))))
    for n in (129, 200, 255, 256):
        cases.append(hash_case("twoblock_len%d" % n, bytes(rng.getrandbits(8) for _ in range(n))))
    for kl, n in ((1, 0), (16, 5), (32, 100), (64, 64)):
        key = bytes(rng.getrandbits(8) for _ in range(kl))
        cases.append(hash_case("keyed_k%d_len%d" % (kl, n),
                               bytes(rng.getrandbits(8) for _ in range(n)), key=key))
    cases.append(hash_case("salt_person", b"hello blake2f", salt=bytes(range(16)),
                           person=b"zk-odst-b2f-mi35"))
    cases.append(hash_case("digest32", b"abc", digest_size=32))
    cases.append(hash_case("abc", b"abc"))

    # The reference's EIP-152 vector (blake2f.rs:196-245), verbatim bytes.
    h1 = bytes.fromhex("48c9bdf267e6096a3ba7ca8485ae67bb2bf894fe72f36e3cf1361d5f3af54fa5")
    h2 = bytes.fromhex("d182e6ad7f520e511f6c3e2b8c68059b6bbd41fbabd9831f79217e1319cde05b")
    m = bytes.fromhex("6162630000000000000000000000000000000000000000000000000000000000") + bytes(96)
    kat = {"name": "reference_eip152_kat", "rounds": 12, "h": hexw(words(h1 + h2, 8)),
           "m": hexw(words(m, 16)), "t": ["%016x" % 3, "%016x" % 0], "f": 1,
           "expected": ("ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
                        "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923"),
           "source": "blake2f-circuit/src/blake2f.rs:193-247"}
    assert kat["expected"] == hashlib.blake2b(b"abc").hexdigest()

    r0 = []
    for i in range(6):
        h = [rng.getrandbits(64) for _ in range(8)]
        t = [rng.getrandbits(64), rng.getrandbits(64) if i % 2 else 0]
        f = i % 2
        mm = [rng.getrandbits(64) for _ in range(16)]
        r0.append({"name": "rounds0_%d" % i, "rounds": 0, "h": hexw(h), "m": hexw(mm),
                   "t": hexw(t), "f": f, "expected": b"".join(
                       struct.pack("<Q", w) for w in rounds0(h, t, f)).hex()})

    spread_rows = [[0, 0, 0], [0, 1, 1],                                  # :684-685
                   [0, 0xff, 0x5555], [1, 0x100, 0x10000],                # :717-718
                   [1, 0x7fff, 0x15555555]]                               # :720-724
    for _ in range(16):
        w = rng.getrandbits(16)
        spread_rows.append([get_tag(w), w, interleave_u16_with_zeros(w)])
    for tag, dense, spread in spread_rows:
        assert spread == spread16(dense) and tag == get_tag(dense)

    out = {"generator": "tests/golden/make_golden.py", "hash_cases": cases, "kat": kat,
           "rounds0": r0, "spread_rows": spread_rows}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "blake2f_golden.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path, len(cases), "hash cases")


if __name__ == "__main__":
    main()
