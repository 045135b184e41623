"""Build the Reuters-21578 views of BASELINE config 3 from the
SGML corpus, restating dataset/reuters/data pre-process.R:7-108 (run here,
where /root/reference exists; the GPU box loads the committed output).

    python scripts/reuters_build.py [--src DIR] [--out FILE]

What the R script does, and how it is restated (the R packages tm / XML are
absent here, so this is a restatement, "parity unpinned" against tm itself):
  * :30-39  read every reut2-*.sgm, split on "</REUTERS>", keep chunks that
    contain "<REUTERS";
  * :9-26   per document: NEWID, the text between <TITLE> and </TITLE>, the
    text between <BODY> and </BODY> (R's sub with a greedy prefix: the last
    such element; "." matches newlines), and ALL <D>...</D> values of the
    document (TOPICS, PLACES, PEOPLE, ORGS, EXCHANGES all use <D>) joined by
    ","; a missing title / body is NA, which tm reads as the text "NA";
  * :50-66  body view: tolower, removePunctuation ([[:punct:]]), removeNumbers
    ([[:digit:]]), removeWords(stopwords("en")) (tm's 174-word English list),
    stripWhitespace; DocumentTermMatrix with terms of >= 3 characters that
    occur in >= 5 documents; counts;
  * :69-85  title view: the same with >= 3 documents;
  * :88-102 topics view: a binary document x value matrix over the sorted
    distinct <D> values.
Output (npz, ~MB): the three count matrices in CSR form (terms sorted, as tm
sorts them), and the documents' TOPICS lists for the ARI truth (mvc_amd.reuters).
"""
import argparse
import glob
import os
import re
import string

import numpy as np

STOPWORDS_EN = """i me my myself we our ours ourselves you your yours yourself yourselves he him his himself she her
hers herself it its itself they them their theirs themselves what which who whom this that these those am is are was
were be been being have has had having do does did doing would should could ought i'm you're he's she's it's we're
they're i've you've we've they've i'd you'd he'd she'd we'd they'd i'll you'll he'll she'll we'll they'll isn't aren't
wasn't weren't hasn't haven't hadn't doesn't don't didn't won't wouldn't shan't shouldn't can't cannot couldn't
mustn't let's that's who's what's here's there's when's where's why's how's a an the and but if or because as until
while of at by for with about against between into through during before after above below to from up down in out
on off over under again further then once here there when where why how all any both each few more most other some
such no nor not only own same so than too very""".split()
assert len(STOPWORDS_EN) == 174

_PUNCT = re.compile("[" + re.escape(string.punctuation) + "]+")
_DIGITS = re.compile("[0-9]+")
_TITLE = re.compile(r".*<TITLE>(.*?)</TITLE>", re.S)
_BODY = re.compile(r".*<BODY>(.*?)</BODY>", re.S)
_D = re.compile(r"<D>(.*?)</D>", re.S)
_TOPICS = re.compile(r"<TOPICS>(.*?)</TOPICS>", re.S)
_NEWID = re.compile(r'NEWID="([0-9]+)"')


def read_docs(src):
    docs = []
    for f in sorted(glob.glob(os.path.join(src, "*.sgm"))):
        with open(f, encoding="latin-1") as fh:
            raw = fh.read()
        for d in raw.split("</REUTERS>"):
            if "<REUTERS" not in d:
                continue
            t = _TITLE.match(d)
            b = _BODY.match(d)
            tp = _TOPICS.search(d)
            docs.append({
                "id": int(_NEWID.search(d).group(1)),
                "title": t.group(1) if t else "NA",
                "body": b.group(1) if b else "NA",
                "d": _D.findall(d),
                "topics": _D.findall(tp.group(1)) if tp else [],
            })
    return docs


def clean(text):
    """tm_map chain of data pre-process.R:52-56, then tokens (words())."""
    x = text.lower()
    x = _PUNCT.sub("", x)
    x = _DIGITS.sub("", x)
    stop = set(STOPWORDS_EN)
    return [w for w in x.split() if w not in stop]


def dtm(texts, min_df):
    """DocumentTermMatrix(control = list(wordLengths = c(3, Inf),
    bounds = list(global = c(min_df, Inf)))): CSR counts, terms sorted."""
    toks = [[w for w in clean(t) if len(w) >= 3] for t in texts]
    df = {}
    for ts in toks:
        for w in set(ts):
            df[w] = df.get(w, 0) + 1
    vocab = sorted(w for w, c in df.items() if c >= min_df)
    col = {w: j for j, w in enumerate(vocab)}
    indptr, indices, data = [0], [], []
    for ts in toks:
        cnt = {}
        for w in ts:
            j = col.get(w)
            if j is not None:
                cnt[j] = cnt.get(j, 0) + 1
        for j in sorted(cnt):
            indices.append(j)
            data.append(cnt[j])
        indptr.append(len(indices))
    return (np.array(indptr, np.int64), np.array(indices, np.int32), np.array(data, np.uint16)), vocab


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="/root/reference/dataset/reuters/reuters21578")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "multiview-clustering_amd", "mvc_amd", "reuters_counts.npz"))
    a = ap.parse_args()
    docs = read_docs(a.src)
    (bp, bi, bd), bv = dtm([d["body"] for d in docs], 5)
    (tp, ti, td), tv = dtm([d["title"] for d in docs], 3)
    dvocab = sorted({x for d in docs for x in d["d"] if x != ""})
    dcol = {x: j for j, x in enumerate(dvocab)}
    kp, ki = [0], []
    for d in docs:
        ki.extend(sorted({dcol[x] for x in d["d"] if x != ""}))
        kp.append(len(ki))
    tvocab = sorted({x for d in docs for x in d["topics"]})
    tcol = {x: j for j, x in enumerate(tvocab)}
    lp, li = [0], []
    for d in docs:
        li.extend(tcol[x] for x in d["topics"])
        lp.append(len(li))
    np.savez_compressed(
        a.out,
        ids=np.array([d["id"] for d in docs], np.int32),
        body_indptr=bp, body_indices=bi, body_data=bd, body_terms=np.array(len(bv)),
        title_indptr=tp, title_indices=ti, title_data=td, title_terms=np.array(len(tv)),
        topics_indptr=np.array(kp, np.int64), topics_indices=np.array(ki, np.int32), topics_terms=np.array(len(dvocab)),
        label_indptr=np.array(lp, np.int64), label_indices=np.array(li, np.int32),
        label_names=np.array(tvocab), topics_names=np.array(dvocab))
    print(f"{len(docs)} documents; body {len(bv)} terms ({bi.size} nonzeros), title {len(tv)} terms, "
          f"<D> values {len(dvocab)}, TOPICS values {len(tvocab)} -> {a.out} ({os.path.getsize(a.out) / 1e6:.1f} MB)")


if __name__ == "__main__":
    main()
