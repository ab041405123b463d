"""Fernet tokens (the format of `cryptography.fernet`) in the standard library only.

The reference's `SecureConfig` (pilott/core/config.py:10-38) stores secrets as Fernet
tokens under a Fernet key file. `cryptography` is not importable in this image, so this
module implements the published Fernet spec directly, which keeps key files and tokens
interchangeable with the reference in both directions:

    key   = urlsafe_b64(signing_key[16] | encryption_key[16])
    token = urlsafe_b64(0x80 | timestamp_be64 | iv[16] | AES-128-CBC(PKCS7(msg)) | HMAC-SHA256[32])

The HMAC covers every byte before it and is checked (constant time) before any
decryption. AES-128 is a plain FIPS-197 implementation; its S-box is derived from the
GF(2^8) inverse at import rather than pasted as a table. Config values are short, so
speed is irrelevant here. Checked against the FIPS-197 known answer and the Fernet spec's
published token (tests/test_core.py).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import struct
import time
from typing import List, Optional, Tuple

__all__ = ["Fernet", "InvalidToken"]


class InvalidToken(Exception):
    """Raised for a malformed, tampered-with or expired token."""


# ---------------------------------------------------------------------------- AES-128
def _xtime(a: int) -> int:
    a <<= 1
    return (a ^ 0x1B) & 0xFF if a & 0x100 else a


def _gmul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = _xtime(a)
        b >>= 1
    return r


def _build_sbox() -> Tuple[List[int], List[int]]:
    inv = [0] * 256
    for a in range(1, 256):
        for b in range(1, 256):
            if _gmul(a, b) == 1:
                inv[a] = b
                break
    sbox = [0] * 256
    for a in range(256):
        x = inv[a]
        y = x
        for _ in range(4):  # affine transform: x ^ rotl(x,1) ^ rotl(x,2) ^ rotl(x,3) ^ rotl(x,4) ^ 0x63
            x = ((x << 1) | (x >> 7)) & 0xFF
            y ^= x
        sbox[a] = y ^ 0x63
    isbox = [0] * 256
    for a, s in enumerate(sbox):
        isbox[s] = a
    return sbox, isbox


_SBOX, _ISBOX = _build_sbox()
_MUL = {c: [_gmul(x, c) for x in range(256)] for c in (2, 3, 9, 11, 13, 14)}


def _expand_key(key: bytes) -> List[List[int]]:
    """11 round keys of 16 bytes (AES-128)."""
    w = [list(key[4 * i:4 * i + 4]) for i in range(4)]
    rcon = 1
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = [_SBOX[b] for b in t[1:] + t[:1]]
            t[0] ^= rcon
            rcon = _xtime(rcon)
        w.append([a ^ b for a, b in zip(w[i - 4], t)])
    return [sum(w[4 * r:4 * r + 4], []) for r in range(11)]


def _shift_rows(s: List[int], inverse: bool = False) -> List[int]:
    # state is column-major: byte (row r, column c) at index 4c + r
    d = -1 if inverse else 1
    return [s[4 * ((c + d * r) % 4) + r] for c in range(4) for r in range(4)]


def _mix_columns(s: List[int], inverse: bool = False) -> List[int]:
    m = ((14, 11, 13, 9), (9, 14, 11, 13), (13, 9, 14, 11), (11, 13, 9, 14)) if inverse else \
        ((2, 3, 1, 1), (1, 2, 3, 1), (1, 1, 2, 3), (3, 1, 1, 2))
    out = []
    for c in range(4):
        col = s[4 * c:4 * c + 4]
        for r in range(4):
            v = 0
            for k in range(4):
                f = m[r][k]
                v ^= col[k] if f == 1 else _MUL[f][col[k]]
            out.append(v)
    return out


def _encrypt_block(rk: List[List[int]], block: bytes) -> bytes:
    s = [b ^ k for b, k in zip(block, rk[0])]
    for r in range(1, 11):
        s = _shift_rows([_SBOX[b] for b in s])
        if r < 10:
            s = _mix_columns(s)
        s = [b ^ k for b, k in zip(s, rk[r])]
    return bytes(s)


def _decrypt_block(rk: List[List[int]], block: bytes) -> bytes:
    s = [b ^ k for b, k in zip(block, rk[10])]
    for r in range(9, -1, -1):
        s = [_ISBOX[b] for b in _shift_rows(s, inverse=True)]
        s = [b ^ k for b, k in zip(s, rk[r])]
        if r > 0:
            s = _mix_columns(s, inverse=True)
    return bytes(s)


def aes128_encrypt_block(key: bytes, block: bytes) -> bytes:
    """One AES-128 block (FIPS-197); exposed for the known-answer test."""
    return _encrypt_block(_expand_key(key), block)


def _cbc_encrypt(key: bytes, iv: bytes, data: bytes) -> bytes:
    rk = _expand_key(key)
    pad = 16 - len(data) % 16
    data += bytes([pad]) * pad
    out, prev = bytearray(), iv
    for i in range(0, len(data), 16):
        prev = _encrypt_block(rk, bytes(a ^ b for a, b in zip(data[i:i + 16], prev)))
        out += prev
    return bytes(out)


def _cbc_decrypt(key: bytes, iv: bytes, data: bytes) -> bytes:
    if not data or len(data) % 16:
        raise InvalidToken("ciphertext is not a whole number of blocks")
    rk = _expand_key(key)
    out, prev = bytearray(), iv
    for i in range(0, len(data), 16):
        blk = data[i:i + 16]
        out += bytes(a ^ b for a, b in zip(_decrypt_block(rk, blk), prev))
        prev = blk
    pad = out[-1]
    if not 1 <= pad <= 16 or out[-pad:] != bytes([pad]) * pad:
        raise InvalidToken("bad padding")
    return bytes(out[:-pad])


# ---------------------------------------------------------------------------- Fernet
class Fernet:
    """`cryptography.fernet.Fernet`'s interface: generate_key, encrypt, decrypt(ttl)."""

    _MAX_CLOCK_SKEW = 60

    def __init__(self, key):
        if isinstance(key, str):
            key = key.encode()
        try:
            raw = base64.urlsafe_b64decode(key)
        except Exception as e:  # noqa: BLE001
            raise ValueError("Fernet key must be 32 url-safe base64-encoded bytes.") from e
        if len(raw) != 32:
            raise ValueError("Fernet key must be 32 url-safe base64-encoded bytes.")
        self._signing_key, self._encryption_key = raw[:16], raw[16:]

    @classmethod
    def generate_key(cls) -> bytes:
        return base64.urlsafe_b64encode(os.urandom(32))

    def encrypt(self, data: bytes) -> bytes:
        return self.encrypt_at_time(data, int(time.time()))

    def encrypt_at_time(self, data: bytes, current_time: int, iv: Optional[bytes] = None) -> bytes:
        iv = os.urandom(16) if iv is None else bytes(iv)
        body = b"\x80" + struct.pack(">Q", current_time) + iv + _cbc_encrypt(self._encryption_key, iv, bytes(data))
        return base64.urlsafe_b64encode(body + hmac.new(self._signing_key, body, hashlib.sha256).digest())

    def decrypt(self, token, ttl: Optional[int] = None) -> bytes:
        return self.decrypt_at_time(token, ttl, int(time.time())) if ttl is not None else self._decrypt(token, None, 0)

    def decrypt_at_time(self, token, ttl: int, current_time: int) -> bytes:
        return self._decrypt(token, ttl, current_time)

    def _decrypt(self, token, ttl: Optional[int], now: int) -> bytes:
        if isinstance(token, str):
            token = token.encode()
        try:
            raw = base64.urlsafe_b64decode(token)
        except Exception as e:  # noqa: BLE001
            raise InvalidToken("token is not url-safe base64") from e
        if len(raw) < 1 + 8 + 16 + 16 + 32 or raw[0] != 0x80:
            raise InvalidToken("not a Fernet token")
        body, tag = raw[:-32], raw[-32:]
        if not hmac.compare_digest(tag, hmac.new(self._signing_key, body, hashlib.sha256).digest()):
            raise InvalidToken("signature mismatch")
        (ts,) = struct.unpack(">Q", body[1:9])
        if ttl is not None:
            if ts + ttl < now:
                raise InvalidToken("token expired")
            if now + self._MAX_CLOCK_SKEW < ts:
                raise InvalidToken("token from the future")
        return _cbc_decrypt(self._encryption_key, body[9:25], body[25:])
