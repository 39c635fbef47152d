"""CPU: the Tokenizer oracle (oracle.tokenize = [U] ml.feature.Tokenizer, toLowerCase.split("\\s"))
against the known answers of Java's String.split(regex) contract (limit 0: interior empty strings
kept, trailing ones removed, no match → the whole string) and Java's \\s class [ \\t\\n\\x0B\\f\\r].
No reference artifact holds tokenizer output (the reference tokenises with CoreNLP,
LDAClustering.scala:116-139), so these documented-behaviour vectors are what pins it."""
import pytest

from oracle import oracle as O

JAVA_SPLIT_KNOWN = [
    ("a b", ["a", "b"]),
    (" a", ["", "a"]),          # leading positive-width match keeps the empty piece
    ("a  b", ["a", "", "b"]),   # interior empty piece kept
    ("a ", ["a"]),              # trailing empty pieces removed
    ("a \t\n", ["a"]),
    ("", [""]),                 # no match: the input itself
    ("abc", ["abc"]),
    ("   ", []),                # every piece is a trailing empty
    ("\t\n\x0b\f\r ", []),
    ("x\x0by", ["x", "y"]),     # \x0B is in Java's \s
    ("x\u00a0y", ["x\u00a0y"]),  # NBSP is not (no UNICODE_CHARACTER_CLASS)
    ("x\u2003y", ["x\u2003y"]),  # nor EM SPACE
    ("x\x1cy", ["x\x1cy"]),     # nor the FS/GS/RS/US separators Python's str.split would take
]


@pytest.mark.parametrize("text,expected", JAVA_SPLIT_KNOWN)
def test_java_split_known_answers(text, expected):
    assert O.java_split_whitespace(text) == expected


def test_tokenize_lowercases_then_splits():
    assert O.tokenize("Hello  WORLD\tÄrger ÜBER Straße") == ["hello", "", "world", "ärger", "über", "straße"]
    assert O.tokenize("×ÞÀ") == ["×þà"]  # U+00D7 has no lower case
