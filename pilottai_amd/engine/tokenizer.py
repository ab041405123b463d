"""Deterministic Llama-3-sized tokenizer for the on-node engine.

There is no network access to fetch the real Llama-3 tokenizer, and the engine
runs random-init weights, so the framework ships its own vocabulary of exactly
Llama-3's size (128,000 regular + 256 special tokens, same special-token ids):

* ids 0..255            single bytes (every string is encodable)
* JSON / schema pieces  ``{"``, ``", "``, ``"]``, ``"requires_decomposition": `` ...
* words                 prompt-template vocabulary and common English words,
                        with and without a leading space; enum values
* numbers               ``0`` .. ``999``
* fillers               seeded pseudo-words up to 128,000 entries
* 128000..128255        ``<|begin_of_text|>``, ``<|end_of_text|>``,
                        ``<|start_header_id|>`` (128006), ``<|end_header_id|>``
                        (128007), ``<|eot_id|>`` (128009), reserved tokens

Encoding is greedy longest-match in the native runtime (csrc/runtime/tokenizer.cpp).
A real HF tokenizer can be plugged in with ``HFTokenizerAdapter`` when one is
available locally.
"""
from __future__ import annotations

import functools
import random
import re
from pathlib import Path
from typing import Iterable, List, Optional, Sequence

import yaml

VOCAB_SIZE = 128256
NUM_REGULAR = 128000
BOS_ID = 128000
EOT_TEXT_ID = 128001  # <|end_of_text|>
START_HEADER_ID = 128006
END_HEADER_ID = 128007
EOT_ID = 128009  # <|eot_id|>

_SPECIAL_NAMES = {
    128000: "<|begin_of_text|>",
    128001: "<|end_of_text|>",
    128006: "<|start_header_id|>",
    128007: "<|end_header_id|>",
    128008: "<|eom_id|>",
    128009: "<|eot_id|>",
    128010: "<|python_tag|>",
}

_COMMON_WORDS = """
the of and to in is that for it as was with be by on not he this are or his from at which but
have an they you were her one all we can there been if more when will would who so no she other
its may these about into than them could only then some time two also after first new most
over such our years like used any what me him well each many much just very where through back
even most state made work make between both being under never day same another know while last
might us great old year off come since against go came right take three states himself few
house use during without again place around however home small found thought went say part once
general high upon school every don does got united left number course war until always away
something fact though water less public put think almost hand enough far took head yet government
system better set told nothing night end why called didn eyes find going look asked later knew
point next program city business give group toward young days let room president side social
given present several order national possible rather second face per among form important often
things looking early white case john become large big need four within felt along children saw
best church ever least power development light thing seemed family interest want members mind
country area others done turned although open god service certain kind problem began different
door thus help sense means whole matter perhaps itself york times law human line above name
example action company hands local show whether five history gave today either act feet across
taken past quite anything having seen death experience body word half really week field car
words already information tell together college shall money period held keep sure probably free
seems political real behind cannot miss question air office making brought whose special major
heard problems federal became study ago moment available known result street economic boy reason
change position south board individual job society areas west close turn love community true
court force full seem am age policy everything including process music room data task tasks agent
agents tool tools result results step steps goal goals role analysis plan execute execution
document documents extract summary summarize evaluate evaluation quality success complete
requirements criteria knowledge memory search query context report text content section
structure review output input value values response format json object list string number
priority complexity dependencies resources estimated minutes hours agents workflow pipeline
manager worker orchestrator delegate delegation load balance scaling fault tolerance health
identify collect verify validate check compute process generate create update store retrieve
key findings insights risks issues improvements actions reasoning alignment challenges
sequence fallback justification assessment outcome validation measurable outcomes
""".split()

_JSON_PIECES = [
    '{"', '"}', '", "', '": "', '": ', ', "', '"]', '["', '[]', '{}', '"', '"}}', '"},', '}}',
    '}, "', '], "', '"], "', '"}, "', ': [', ': {', '": [', '": {', '": ["', '": {"', '", ', ' "',
    '{', '}', '[', ']', ',', ':', ', ', ': ', '\n', '\n\n', '  ', '    ', 'true', 'false', 'null',
    '```', '```json', '\\n', '...', '. ', '.\n', ' -', '- ',
]


@functools.lru_cache(maxsize=1)
def _rules_words() -> List[str]:
    """Words and JSON keys that appear in the prompt rules (source/rules.yaml)."""
    path = Path(__file__).resolve().parent.parent / "source" / "rules.yaml"
    words: List[str] = []
    keys: List[str] = []
    enums: List[str] = []
    if path.exists():
        data = yaml.safe_load(path.read_text())
        text = yaml.safe_dump(data)
        words = re.findall(r"[A-Za-z][A-Za-z_]*", text)

        def walk(node):
            if isinstance(node, dict):
                for k, v in node.items():
                    keys.append(str(k))
                    walk(v)
            elif isinstance(node, str):
                m = re.match(r"enum\((.*)\)", node)
                if m:
                    enums.extend(m.group(1).split("|"))

        for section in ("schemas",):
            walk(data.get(section, {}))
    return sorted(set(words)) + ["__KEYS__"] + sorted(set(keys)) + ["__ENUMS__"] + sorted(set(enums))


def build_vocab(extra_words: Iterable[str] = ()) -> List[bytes]:
    vocab: List[bytes] = [bytes([i]) for i in range(256)]
    seen = set(vocab)

    def add(piece: str):
        b = piece.encode("utf-8")
        if b and b not in seen and len(vocab) < NUM_REGULAR:
            seen.add(b)
            vocab.append(b)

    rw = _rules_words()
    split = rw.index("__KEYS__")
    split2 = rw.index("__ENUMS__")
    words, keys, enums = rw[:split], rw[split + 1:split2], rw[split2 + 1:]
    for p in _JSON_PIECES:
        add(p)
    for k in keys:
        add(f'"{k}": ')
        add(f'{{"{k}": ')
        add(f', "{k}": ')
        add(f'"{k}"')
        add(k)
    for e in enums + ["low", "medium", "high", "critical", "true", "false"]:
        add(e)
        add(f'"{e}"')
    for n in range(1000):
        add(str(n))
    for w in list(_COMMON_WORDS) + list(words) + list(extra_words):
        for form in (w, w.capitalize()):
            add(form)
            add(" " + form)
    rng = random.Random(0x5EED)
    letters = "abcdefghijklmnopqrstuvwxyz"
    while len(vocab) < NUM_REGULAR:
        n = rng.randint(2, 8)
        w = "".join(rng.choice(letters) for _ in range(n))
        add(w if rng.random() < 0.3 else " " + w)
    specials = [f"<|reserved_special_token_{i}|>".encode() for i in range(VOCAB_SIZE - NUM_REGULAR)]
    for tid, name in _SPECIAL_NAMES.items():
        specials[tid - NUM_REGULAR] = name.encode()
    vocab.extend(specials)
    assert len(vocab) == VOCAB_SIZE
    return vocab


def _is_string_safe(piece: bytes) -> bool:
    if not piece:
        return False
    for c in piece:
        if c < 0x20 or c >= 0x80 or c in (0x22, 0x5C):  # control, non-ASCII, quote, backslash
            return False
    return True


class Tokenizer:
    """Native greedy longest-match tokenizer over the Llama-3-sized vocabulary."""

    bos_id = BOS_ID
    eot_id = EOT_ID
    eos_ids = (EOT_TEXT_ID, EOT_ID)

    def __init__(self, vocab: Optional[Sequence[bytes]] = None):
        from pilottai_amd import _runtime

        self.vocab: List[bytes] = list(vocab) if vocab is not None else build_vocab()
        self._native = _runtime.Tokenizer(self.vocab)
        self.vocab_size = len(self.vocab)

    def encode(self, text: str) -> List[int]:
        return self._native.encode(text)

    def decode(self, ids: Sequence[int]) -> str:
        return self._native.decode(list(ids)).decode("utf-8", errors="replace")

    def token_id(self, piece: str) -> int:
        return self._native.lookup(piece.encode("utf-8"))

    def string_safe_mask(self):
        import numpy as np

        m = np.zeros(self.vocab_size, dtype=bool)
        for i, p in enumerate(self.vocab[:NUM_REGULAR]):
            m[i] = _is_string_safe(p)
        return m


@functools.lru_cache(maxsize=1)
def get_tokenizer() -> Tokenizer:
    return Tokenizer()
