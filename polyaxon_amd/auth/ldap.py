"""Minimal LDAPv3 client: simple bind, subtree search, unbind (RFC 4511 BER over TCP).

Reference: ``django_auth_ldap.backend.LDAPBackend`` configured by config_settings/auth.py:10-80
(``POLYAXON_AUTH_LDAP_SERVER_URI``, ``BIND_DN``/``BIND_PASSWORD``, ``USER_SEARCH_BASE_DN`` +
``USER_SEARCH_FILTERSTR``, ``USER_DN_TEMPLATE``, ``USER_ATTR_MAP``).  ``python-ldap`` is not part of this
image, so the handful of protocol operations a login needs are encoded here directly:

* **DN template**: bind as ``user_dn_template.format(username=...)`` with the user's password;
* **search**: bind as the service account, search ``search_base_dn`` with ``search_filter`` (RFC 4515 subset:
  ``(a=v)``, ``(a=*)``, ``(&...)``, ``(|...)``, ``(!...)``), then bind as the DN found.

Assertion values are escaped before they enter the filter, so a username cannot widen the search.
``ldaps://`` wraps the socket in TLS (system trust store).
"""
from __future__ import annotations

import socket
import ssl
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple
from urllib.parse import urlparse

# ---------------------------------------------------------------------------------------------- BER


def _len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def tlv(tag: int, content: bytes) -> bytes:
    return bytes([tag]) + _len(len(content)) + content


def ber_int(v: int, tag: int = 0x02) -> bytes:
    n = max(1, (v.bit_length() + 8) // 8)
    return tlv(tag, v.to_bytes(n, "big", signed=True))


def ber_str(s, tag: int = 0x04) -> bytes:
    return tlv(tag, s.encode() if isinstance(s, str) else bytes(s))


def ber_bool(v: bool) -> bytes:
    return tlv(0x01, b"\xff" if v else b"\x00")


def seq(*items: bytes, tag: int = 0x30) -> bytes:
    return tlv(tag, b"".join(items))


def read_tlv(buf: bytes, off: int = 0) -> Tuple[int, bytes, int]:
    """Return (tag, content, next_offset)."""
    if off + 2 > len(buf):
        raise EOFError
    tag = buf[off]
    n = buf[off + 1]
    off += 2
    if n & 0x80:
        k = n & 0x7F
        if off + k > len(buf):
            raise EOFError
        n = int.from_bytes(buf[off:off + k], "big")
        off += k
    if off + n > len(buf):
        raise EOFError
    return tag, buf[off:off + n], off + n


def children(content: bytes) -> List[Tuple[int, bytes]]:
    out, off = [], 0
    while off < len(content):
        t, c, off = read_tlv(content, off)
        out.append((t, c))
    return out


def as_int(content: bytes) -> int:
    return int.from_bytes(content, "big", signed=True) if content else 0

# ---------------------------------------------------------------------------------------------- filters


def escape_filter_value(v: str) -> str:
    out = []
    for ch in v:
        if ch in "*()\\\x00":
            out.append("\\%02x" % ord(ch))
        else:
            out.append(ch)
    return "".join(out)


def _unescape(v: str) -> bytes:
    out, i = bytearray(), 0
    while i < len(v):
        if v[i] == "\\" and i + 2 < len(v) and all(c in "0123456789abcdefABCDEF" for c in v[i + 1:i + 3]):
            out.append(int(v[i + 1:i + 3], 16))
            i += 3
        else:
            out.extend(v[i].encode())
            i += 1
    return bytes(out)


def encode_filter(f: str) -> bytes:
    node, rest = _parse_filter(f.strip(), 0)
    if rest != len(f.strip()):
        raise ValueError(f"trailing characters in LDAP filter {f!r}")
    return node


def _parse_filter(s: str, i: int) -> Tuple[bytes, int]:
    if i >= len(s) or s[i] != "(":
        raise ValueError(f"LDAP filter: expected '(' at {i} in {s!r}")
    i += 1
    if s[i] in "&|":
        tag = 0xA0 if s[i] == "&" else 0xA1
        i += 1
        parts = []
        while s[i] == "(":
            p, i = _parse_filter(s, i)
            parts.append(p)
        if s[i] != ")":
            raise ValueError("LDAP filter: unbalanced parentheses")
        return tlv(tag, b"".join(parts)), i + 1
    if s[i] == "!":
        p, i = _parse_filter(s, i + 1)
        if s[i] != ")":
            raise ValueError("LDAP filter: unbalanced parentheses")
        return tlv(0xA2, p), i + 1
    j = s.index(")", i)
    item = s[i:j]
    if "=" not in item:
        raise ValueError(f"LDAP filter item without '=': {item!r}")
    attr, val = item.split("=", 1)
    if val == "*":
        return ber_str(attr, 0x87), j + 1
    if "*" in val:
        raise ValueError("LDAP filter: substring matches are not supported")
    return tlv(0xA3, ber_str(attr) + ber_str(_unescape(val))), j + 1

# ---------------------------------------------------------------------------------------------- client


class LDAPError(RuntimeError):
    def __init__(self, code: int, message: str = ""):
        super().__init__(f"LDAP result {code}: {message}")
        self.code = code


INVALID_CREDENTIALS = 49


@dataclass
class Entry:
    dn: str
    attrs: Dict[str, List[str]] = field(default_factory=dict)

    def first(self, name: str) -> Optional[str]:
        for k, v in self.attrs.items():
            if k.lower() == name.lower() and v:
                return v[0]
        return None


class LDAPConnection:
    def __init__(self, uri: str, timeout: float = 5.0):
        u = urlparse(uri)
        if u.scheme not in ("ldap", "ldaps"):
            raise ValueError(f"unsupported LDAP URI {uri!r}")
        port = u.port or (636 if u.scheme == "ldaps" else 389)
        sock = socket.create_connection((u.hostname, port), timeout=timeout)
        if u.scheme == "ldaps":
            sock = ssl.create_default_context().wrap_socket(sock, server_hostname=u.hostname)
        self.sock = sock
        self.msg_id = 0
        self._buf = b""

    def close(self) -> None:
        try:
            self._send(tlv(0x42, b""))  # UnbindRequest (NULL body)
        except OSError:
            pass
        self.sock.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _send(self, op: bytes) -> int:
        self.msg_id += 1
        self.sock.sendall(seq(ber_int(self.msg_id), op))
        return self.msg_id

    def _recv(self) -> Tuple[int, int, bytes]:
        while True:
            try:
                _, content, end = read_tlv(self._buf)
                self._buf = self._buf[end:]
                parts = children(content)
                return as_int(parts[0][1]), parts[1][0], parts[1][1]
            except EOFError:
                chunk = self.sock.recv(65536)
                if not chunk:
                    raise ConnectionError("LDAP server closed the connection")
                self._buf += chunk

    @staticmethod
    def _result(content: bytes) -> None:
        parts = children(content)
        code = as_int(parts[0][1])
        if code != 0:
            raise LDAPError(code, parts[2][1].decode(errors="replace") if len(parts) > 2 else "")

    def bind(self, dn: str, password: str) -> None:
        if not password:  # an empty simple-bind password is an *anonymous* bind (RFC 4513 §5.1.2)
            raise LDAPError(INVALID_CREDENTIALS, "empty password")
        mid = self._send(seq(ber_int(3), ber_str(dn), ber_str(password, 0x80), tag=0x60))
        rid, tag, content = self._recv()
        if rid != mid or tag != 0x61:
            raise LDAPError(-1, f"unexpected response tag 0x{tag:02x}")
        self._result(content)

    def search(self, base: str, filt: str, attrs: List[str], size_limit: int = 2, scope: int = 2) -> List[Entry]:
        """scope: 0 = base object, 1 = one level, 2 = whole subtree."""
        op = seq(ber_str(base), ber_int(scope, 0x0A), ber_int(0, 0x0A), ber_int(size_limit), ber_int(0),
                 ber_bool(False), encode_filter(filt), seq(*[ber_str(a) for a in attrs]), tag=0x63)
        mid = self._send(op)
        out: List[Entry] = []
        while True:
            rid, tag, content = self._recv()
            if rid != mid:
                continue
            if tag == 0x64:  # SearchResultEntry
                parts = children(content)
                e = Entry(parts[0][1].decode())
                for _, pa in children(parts[1][1]):
                    kv = children(pa)
                    e.attrs[kv[0][1].decode()] = [v.decode(errors="replace") for _, v in children(kv[1][1])]
                out.append(e)
            elif tag == 0x65:  # SearchResultDone
                self._result(content)
                return out
            # 0x73 referral: ignored


@dataclass
class LDAPAuthenticator:
    server_uri: str
    user_dn_template: Optional[str] = None
    bind_dn: Optional[str] = None
    bind_password: Optional[str] = None
    search_base_dn: Optional[str] = None
    search_filter: str = "(uid={username})"
    attr_map: Dict[str, str] = field(default_factory=lambda: {"email": "mail"})
    timeout_s: float = 5.0

    @classmethod
    def from_settings(cls, s) -> Optional["LDAPAuthenticator"]:
        if not s.get("auth.ldap.enabled"):
            return None
        return cls(s.get("auth.ldap.server_uri"), s.get("auth.ldap.user_dn_template"), s.get("auth.ldap.bind_dn"),
                   s.get("auth.ldap.bind_password"), s.get("auth.ldap.search_base_dn"),
                   s.get("auth.ldap.search_filter"), s.get("auth.ldap.attr_map"), s.get("auth.ldap.timeout_s"))

    def authenticate(self, username: str, password: str) -> Optional[Dict[str, str]]:
        """Return the mapped user fields on success, None on bad credentials; raise on server errors."""
        if not username or not password:
            return None
        with LDAPConnection(self.server_uri, self.timeout_s) as conn:
            if self.user_dn_template:
                dn = self.user_dn_template.format(username=username)
                entry = Entry(dn)
            else:
                if self.bind_dn:
                    conn.bind(self.bind_dn, self.bind_password or "")
                filt = self.search_filter.format(username=escape_filter_value(username))
                found = conn.search(self.search_base_dn or "", filt, sorted(set(self.attr_map.values())))
                if len(found) != 1:
                    return None
                entry = found[0]
            try:
                conn.bind(entry.dn, password)
            except LDAPError as e:
                if e.code == INVALID_CREDENTIALS:
                    return None
                raise
            if self.user_dn_template and self.attr_map:
                try:
                    hits = conn.search(entry.dn, "(objectClass=*)", sorted(set(self.attr_map.values())), 1, scope=0)
                    if hits:
                        entry = hits[0]
                except LDAPError:
                    pass
        out = {"username": username, "dn": entry.dn}
        for field_name, attr in self.attr_map.items():
            v = entry.first(attr)
            if v is not None:
                out[field_name] = v
        return out
