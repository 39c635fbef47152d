"""Generate the golden fixtures under tests/golden/ from the reference's own artefacts.

Run ONCE in the build container (the only place /root/reference exists):

    python tests/golden/make_golden.py

Nothing at test time reads /root/reference: the tests read only the .npz/.json files this
script writes.  The fixtures are DATA extracted from the reference's saved models and run
logs (inputs and expected outputs), never reference source text.

Fixtures:

F1 ``en_idf.npz`` / ``ge_idf.npz`` — IDF(minDocFreq=2) + 1e-4 floor, pinned bit-exactly.
    Source: ``models/LdaModel_{EN_1591049082850,GE_1591070442475}/data/tokenCounts``.
    Each parquet edge (srcId=doc, dstId=-(term+1), tokenCounts=tf*idf') is the TF·IDF value
    the reference fed to LDA (LDAClustering.scala:177-192).  We recover the integer TF as
    round(value/idf') where idf' is recomputed from the edge incidence, and store the
    integer TF CSR next to the stored TF·IDF values: an IDF implementation is correct iff
    tf*idf' reproduces every stored value bit for bit.
F2 ``en_describe.json`` + ``en_topics.npz`` — describeTopics known answers.
    Source: ``data/topicCounts`` (term vertices, id = -(term+1)) and the printed top terms
    in ``TestOutput/Result_EN_1591066624209:4-51`` and ``Result_EN_1591723228815:1028-1150``.
F3 ``en_topicdist.json`` — LocalLDAModel.topicDistribution known answers: the 51 books × 5
    topic proportions printed by LDALoader.scala:108-135 in both Result files (two
    independent runs: their spread is the fixture's noise floor).
F4 metadata (α, η, k, gammaShape) from ``metadata/part-00000`` is copied into the json.
F5 ``en_vocab.txt`` and F6 ``books_text.json`` — see make_vocab / make_text_samples.
"""
import glob
import json
import os
import re
import sys

import numpy as np

REF = "/root/reference/TextClustering/src/main/resources"
OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))


def _read_table(d):
    import pyarrow.parquet as pq
    import pyarrow as pa
    fs = sorted(glob.glob(os.path.join(d, "*.parquet")))
    return pa.concat_tables([pq.read_table(f) for f in fs])


def _edges(model):
    t = _read_table(os.path.join(REF, "models", model, "data", "tokenCounts"))
    src = t.column("srcId").to_numpy().astype(np.int64)
    dst = t.column("dstId").to_numpy().astype(np.int64)
    val = t.column("tokenCounts").to_numpy().astype(np.float64)
    term = -(dst + 1)
    assert (term >= 0).all() and (src >= 0).all()
    return src, term, val


def make_idf(model, tag):
    meta = json.load(open(os.path.join(REF, "models", model, "metadata", "part-00000")))
    V = int(meta["vocabSize"])
    doc, term, val = _edges(model)
    order = np.lexsort((term, doc))
    doc, term, val = doc[order], term[order], val[order]
    # doc ids come from zipWithIndex *before* the empty-doc filter (LDAClustering.scala:132-139),
    # so they may have gaps: IDF's m counts the surviving docs, i.e. the distinct ids.
    doc_ids, doc = np.unique(doc, return_inverse=True)
    m = int(doc_ids.size)
    # df and the reference's floored idf (LDAClustering.scala:177-188; mllib IDF.idf)
    df = np.bincount(term, minlength=V).astype(np.int64)
    idf = np.where(df >= 2, np.log((m + 1.0) / (df + 1.0)), 0.0)
    idf_f = np.where(idf == 0.0, 1e-4, idf)
    tf_real = val / idf_f[term]
    tf = np.rint(tf_real)
    dev = float(np.abs(tf_real - tf).max())
    assert dev < 1e-9, dev
    tf = tf.astype(np.int32)
    assert (tf >= 1).all()
    assert np.array_equal(tf * idf_f[term], val), "recovered TF must reproduce the edges exactly"
    indptr = np.zeros(m + 1, np.int64)
    np.cumsum(np.bincount(doc, minlength=m), out=indptr[1:])
    np.savez_compressed(
        os.path.join(OUT, f"{tag}_idf.npz"),
        indptr=indptr, indices=term.astype(np.int32), tf=tf, tfidf=val, doc_ids=doc_ids,
        num_docs=np.int64(m), vocab_size=np.int64(V), min_doc_freq=np.int64(2))
    print(f"{tag}: m={m} V={V} nnz={val.size} tokens={int(tf.sum())} max|tf-round|={dev:.2e}")
    return indptr, term.astype(np.int32), tf, meta


def _topic_counts(model, V, k):
    t = _read_table(os.path.join(REF, "models", model, "data", "topicCounts")).to_pylist()
    nwk = np.zeros((V, k), np.float64)
    seen = 0
    for row in t:
        vid = row["id"]
        if vid < 0:
            tw = row["topicWeights"]
            assert tw["type"] == 1
            nwk[-(vid + 1)] = tw["values"]
            seen += 1
    assert seen == V
    g = _read_table(os.path.join(REF, "models", model, "data", "globalTopicTotals")).to_pylist()
    totals = np.array(g[0]["globalTopicTotals"]["values"], np.float64)
    return nwk, totals


def _parse_topics(path, first_line, last_line):
    """Parse 'TOPIC i' blocks with 'term\\tweight' lines between the given 1-based lines."""
    lines = open(path, encoding="utf-8").read().split("\n")[first_line - 1:last_line]
    topics, cur = {}, None
    for ln in lines:
        mt = re.match(r"TOPIC (\d+)", ln)
        if mt:
            cur = int(mt.group(1))
            topics[cur] = []
            continue
        if cur is not None and "\t" in ln:
            term, w = ln.split("\t")
            topics[cur].append((term, w))
    return topics


def _parse_distributions(path):
    txt = open(path, encoding="utf-8").read()
    blocks = txt.split("Book's number: ")[1:]
    out = []
    for b in blocks:
        name = re.search(r"Book's name: (.*)", b).group(1)
        ws = re.findall(r"Nr\.: (\d+) \t\t\|\t (\S+)", b)
        out.append({"book": name, "dist": [w for _, w in ws]})
    return out


def make_en_model_fixtures(indptr, indices, tf, meta):
    model = "LdaModel_EN_1591049082850"
    k, V = int(meta["k"]), int(meta["vocabSize"])
    nwk, totals = _topic_counts(model, V, k)
    vocab = open(os.path.join(REF, "models", "vocabularies", model), encoding="utf-8").read().split(",")
    assert len(vocab) == V
    np.savez_compressed(os.path.join(OUT, "en_topics.npz"), nwk=nwk, totals=totals)

    r1 = os.path.join(REF, "TestOutput", "Result_EN_1591066624209")
    r2 = os.path.join(REF, "TestOutput", "Result_EN_1591723228815")
    # Result_EN_1591066624209:4-51 (top-8 per topic); Result_EN_1591723228815:1028-1150 (top-10)
    t1 = _parse_topics(r1, 4, 51)
    t2 = _parse_topics(r2, 1020, 1150)
    term_index = {}
    for i, w in enumerate(vocab):
        term_index.setdefault(w, i)
    describe = {}
    for name, tops in (("Result_EN_1591066624209", t1), ("Result_EN_1591723228815", t2)):
        describe[name] = {
            str(t): [{"term": w, "index": term_index[w], "weight": s} for w, s in lst]
            for t, lst in tops.items()}
    d1 = _parse_distributions(r1)
    d2 = _parse_distributions(r2)
    assert len(d1) == len(d2) == indptr.size - 1
    dist = {"books": [x["book"] for x in d2],
            "Result_EN_1591066624209": [x["dist"] for x in d1],
            "Result_EN_1591723228815": [x["dist"] for x in d2]}
    common = {"model": model, "k": k, "vocab_size": V,
              "docConcentration": meta["docConcentration"],
              "topicConcentration": meta["topicConcentration"],
              "gammaShape": meta["gammaShape"]}
    json.dump({**common, "describe": describe}, open(os.path.join(OUT, "en_describe.json"), "w"),
              indent=1)
    json.dump({**common, **dist}, open(os.path.join(OUT, "en_topicdist.json"), "w"), indent=1)
    print("describe/topicdist fixtures written")


def make_vocab():
    """F5 ``en_vocab.txt`` — the EN model's vocabulary (vocabArray, index = term id, one per line), the
    strings behind en_idf.npz's term ids: the config-1 pipeline test hashes them (HashingTF)."""
    model = "LdaModel_EN_1591049082850"
    vocab = open(os.path.join(REF, "models", "vocabularies", model), encoding="utf-8").read().split(",")
    assert all("\n" not in w for w in vocab)
    with open(os.path.join(OUT, "en_vocab.txt"), "w", encoding="utf-8") as f:
        f.write("\n".join(vocab) + "\n")
    print(f"en_vocab.txt: {len(vocab)} terms")


# the lines of the reference's books that the round-2 kernel rejected (Greek Extended, U+2116 "№"):
# one slice around each goes into the fixture as well
TARGET_LINES = [("English", "Walden - Henry David Thoreau.txt", 1593),
                ("Russian", "2012 20 eink - Unknown.txt", 141),
                ("Russian", "Adiutant iegho prievoskhoditiel'stva - Vladimir Galaktionovich Korolienko.txt", 14),
                ("Russian", "Stat'i ob okhotie - Sierghiei Timofieievich Aksakov.txt", 15),
                ("Ukrainian", "Ia (Romantika) - Mikola Khvil'ovii.txt", 308)]


def make_text_samples(per_lang=3, width=2500):
    """F6 ``books_text.json`` — raw text slices of the reference's own corpora (resources/books/<Lang>):
    three books per language, ``width`` characters from a third of the way in, plus one slice around
    each line of TARGET_LINES (key "targets").  No slice is moved or filtered: the tokenizer's lower-casing
    tests take the text as it is."""
    out = {}
    base = os.path.join(REF, "books")
    for lang in sorted(os.listdir(base)):
        books = sorted(os.listdir(os.path.join(base, lang)))[:per_lang]
        samples = []
        for b in books:
            t = open(os.path.join(base, lang, b), encoding="utf-8").read()
            p = len(t) // 3
            samples.append({"book": b, "offset": p, "text": t[p:p + width]})
        out[lang] = samples
    targets = []
    for lang, b, line in TARGET_LINES:
        t = open(os.path.join(base, lang, b), encoding="utf-8").read()
        lines = t.split("\n")
        p = len("\n".join(lines[:line - 1])) + 1  # the line's first character (1-based line numbers)
        # centred on the line's first character past U+0FFF (the Greek Extended letter, the "№")
        q = next(i for i in range(p, p + len(lines[line - 1])) if ord(t[i]) > 0xFFF)
        lo = max(0, q - width // 2)
        targets.append({"book": f"{lang}/{b}", "line": line, "offset": lo, "text": t[lo:lo + width]})
    out["targets"] = targets
    json.dump(out, open(os.path.join(OUT, "books_text.json"), "w", encoding="utf-8"), ensure_ascii=False, indent=0)
    print("books_text.json:", {k: len(v) for k, v in out.items()})


def check_all_books():
    """Every character of every book under resources/books is one the tokenizer kernel accepts (the
    generated case table's rejects: tools/gen_case_table.py).  Prints the count; raises otherwise."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_case_table as g

    idx, data = g.pages()
    rejected = {(idx.index(pi + 1) << 8) + i for pi, ent in enumerate(data) for i, e in enumerate(ent) if e == 0} - {0}
    base = os.path.join(REF, "books")
    n = 0
    for lang in sorted(os.listdir(base)):
        for b in sorted(os.listdir(os.path.join(base, lang))):
            t = open(os.path.join(base, lang, b), encoding="utf-8").read()
            bad = sorted({hex(ord(c)) for c in t if ord(c) in rejected})
            assert not bad, (lang, b, bad)
            n += 1
    print(f"all {n} books: every character accepted by the tokenizer kernel")


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference not present: fixtures are generated only in the build container")
    if sys.argv[1:] == ["--text"]:  # the F5/F6 fixtures only (the npz files stay byte-identical)
        make_vocab()
        make_text_samples()
        check_all_books()
        sys.exit(0)
    ip, ix, tf, meta = make_idf("LdaModel_EN_1591049082850", "en")
    make_idf("LdaModel_GE_1591070442475", "ge")
    make_en_model_fixtures(ip, ix, tf, meta)
    make_vocab()
    make_text_samples()
