"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

``make asan`` (bayesian-consensus-engine_amd/csrc, oracle) builds two harness executables with
-fsanitize=address,undefined: tests/native/jsonl_fuzz.cpp drives the JSONL front end
(csrc/jsonl.cpp: parse on 1..4 threads, arrays, render) over a corpus of the golden CLI and
validation payloads plus a seeded set of mutations (truncations, byte flips, deep nesting, huge
numbers, lone surrogates, duplicate keys, control bytes, long ids); tests/native/oracle_fuzz.c
drives every entry point of the C restatement over random batches.  Any sanitizer report fails
the run (-fno-sanitize-recover, halt_on_error)."""
import json
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
JSONL_FUZZ = os.path.join(ROOT, "bayesian-consensus-engine_amd", "lib", "asan", "jsonl_fuzz")
ORACLE_FUZZ = os.path.join(ROOT, "oracle", "_build", "asan", "oracle_fuzz")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "bayesian-consensus-engine_amd", "csrc"), "asan"],
                   check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)


def _seeds():
    out = []
    cli = json.load(open(os.path.join(GOLD, "cli_cases.json")))
    for v in cli["inputs"].values():
        out.append(json.dumps(v) if not isinstance(v, str) else v.replace("\n", " "))
    for c in json.load(open(os.path.join(GOLD, "validate_cases.json"))):
        out.append(json.dumps(c["payload"]))
    rng = random.Random(3)
    for i in range(60):
        sig = [{"sourceId": f"s{rng.randrange(40)}", "probability": rng.random()} for _ in range(rng.randrange(0, 50))]
        out.append(json.dumps({"schemaVersion": "1.0.0", "marketId": f"m{i}", "signals": sig}))
    return out


def _mutate(s: str, rng: random.Random) -> str:
    k = rng.randrange(12)
    if k == 0 and s:
        return s[:rng.randrange(len(s))]                                         # truncation
    if k == 1 and s:
        i = rng.randrange(len(s))
        return s[:i] + chr(rng.choice([0x22, 0x5C, 0x7B, 0x7D, 0x5B, 0x5D, 0x2C, 0x3A, 0x01, 0x7F])) + s[i + 1:]
    if k == 2:
        d = rng.randrange(200, 5000)
        return "[" * d + "]" * d                                                # deep nesting
    if k == 3:
        return s.replace('"probability": 0', '"probability": 1e400', 1).replace("0.", "1e-400", 1)
    if k == 4:
        return s.replace('"s', '"\\ud800s', 1)                                  # lone surrogate
    if k == 5:
        return s.replace('"marketId"', '"marketId": 1, "marketId"', 1)          # duplicate key
    if k == 6:
        return s.replace('"s', '"' + "\\u00e9\\uD83D\\uDE00" * rng.randrange(1, 50) + "s", 1)
    if k == 7:
        return s.replace('"s', '"' + "x" * rng.randrange(1000, 20000), 1)     # long id
    if k == 8:
        return s.replace("0.", "NaN, \"x\": Infinity, \"y\": -Infinity, \"z\": 0.", 1)
    if k == 9:
        return s.replace('"probability"', '"probability": true, "p"', 1)
    if k == 10:
        return "   \t" + s + "  \r"
    return s.replace("1.0.0", "1.0.1", 1)


def _corpus(n_mut=3000):
    rng = random.Random(7)
    seeds = _seeds()
    lines = list(seeds)
    for _ in range(n_mut):
        s = rng.choice(seeds)
        for _ in range(rng.randrange(1, 4)):
            s = _mutate(s, rng)
        lines.append(s.replace("\n", " "))
    return "\n".join(lines) + "\n"


@pytest.mark.timeout(600)
def test_jsonl_front_end_under_asan_ubsan(tmp_path):
    _build()
    p = tmp_path / "corpus.jsonl"
    p.write_text(_corpus(), encoding="utf-8", errors="surrogatepass")
    r = subprocess.run([JSONL_FUZZ, str(p)], capture_output=True, text=True, env=ENV, timeout=500)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "jsonl_fuzz ok" in r.stdout


@pytest.mark.timeout(600)
def test_oracle_restatement_under_asan_ubsan():
    _build()
    r = subprocess.run([ORACLE_FUZZ, "40"], capture_output=True, text=True, env=ENV, timeout=500)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "oracle_fuzz ok" in r.stdout
