"""Bucket statistics of the match finder's hash4 buckets per 256 KiB stream (CPU, numpy).

For VERDICT r05 next-5 (TEXT walk): how the members spread over bucket-length classes, how many
members of long buckets (>= 256) are 'replacements' (LCP with the previous member of the bucket
>= fb, so BinTree.java:246-252 ends their walk at the first node and they inherit its children),
and the tree steps per member of a BinTree insertion (BinTree.java:228-270, cut_value and
len_limit as level 5 fb 32), simulated on one stream per data kind.

Buckets are grouped by the four bytes themselves (hash4 with 24 - 26 bits only adds rare
collisions). Usage: python tools/r06/text_buckets.py [streams]
"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "..", "lzma-java_amd"))
import lzma_amd  # noqa: E402

S = 262144
FB = 32
CUT = 16 + FB // 2


def buckets(b):
    k = b[:-3] | (b[1:-2] << 8) | (b[2:-1] << 16) | (b[3:] << 24)
    order = np.argsort(k, kind="stable")
    ks = k[order]
    heads = np.r_[True, ks[1:] != ks[:-1]]
    starts = np.nonzero(heads)[0]
    lens = np.diff(np.r_[starts, len(ks)])
    return order, heads, lens


def class_stats(kind, nstreams):
    d = lzma_amd.generate(kind, S * nstreams)
    hist, longest = {}, []
    long_members = long_rep = 0
    for s in range(nstreams):
        b = d[s * S:(s + 1) * S].astype(np.uint32)
        order, heads, lens = buckets(b)
        longest.append(int(lens.max()))
        for L in lens:
            c = 1 << int(np.log2(L))
            hist[c] = hist.get(c, 0) + int(L)
        prevp = np.r_[-1, order[:-1]]
        prevp[heads] = -1
        blen = np.repeat(lens, lens)
        m = (prevp >= 0) & (order + FB <= S) & (blen >= 256)
        p, q = order[m], prevp[m]
        eq = np.ones(len(p), bool)
        for j in range(FB):
            eq &= b[p + j] == b[q + j]
        long_members += int((blen >= 256).sum())
        long_rep += int(eq.sum())
    return hist, longest, long_members, long_rep


def walk_steps(kind):
    """Tree steps per member of one stream's BinTree insertions, by bucket-length class."""
    b = bytes(lzma_amd.generate(kind, S)[:S])
    order, heads, lens = buckets(np.frombuffer(b, np.uint8).astype(np.uint32))
    bucket_len = np.repeat(lens, lens)
    cls_of = {int(order[i]): int(bucket_len[i]) for i in range(len(order))}
    son = {}
    head = {}
    steps_by = {}
    n = len(b)
    for p in range(n - 3):
        key = b[p:p + 4]
        cur = head.get(key)
        head[key] = p
        lim = min(FB, n - p)
        ptr0, ptr1 = (p, 1), (p, 0)
        len0 = len1 = 0
        count = CUT
        steps = 0
        while True:
            if cur is None or count == 0:
                son[ptr0] = None
                son[ptr1] = None
                break
            count -= 1
            steps += 1
            ln = min(len0, len1)
            while ln < lim and b[cur + ln] == b[p + ln]:
                ln += 1
            if ln == lim:
                son[ptr1] = son.get((cur, 0))
                son[ptr0] = son.get((cur, 1))
                break
            if b[cur + ln] < b[p + ln]:
                son[ptr1] = cur
                ptr1 = (cur, 1)
                len1 = ln
                cur = son.get((cur, 1))
            else:
                son[ptr0] = cur
                ptr0 = (cur, 0)
                len0 = ln
                cur = son.get((cur, 0))
        c = 1 << int(np.log2(cls_of[p]))
        t = steps_by.setdefault(c, [0, 0])
        t[0] += 1
        t[1] += steps
    return steps_by


def main():
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    for kind in ("text", "bench"):
        hist, longest, lm, lr = class_stats(kind, ns)
        tot = sum(hist.values())
        print("%s: %d streams of 256 KiB, %d members" % (kind, ns, tot))
        print("  members by bucket-length class: " + ", ".join("%d: %.1f%%" % (c, 100.0 * v / tot) for c, v in sorted(hist.items())))
        print("  longest bucket per stream: median %d, max %d" % (int(np.median(longest)), max(longest)))
        print("  members of buckets >= 256: %d (%.1f%%); replacements (LCP with the previous member >= %d): %d"
              % (lm, 100.0 * lm / tot, FB, lr))
        st = walk_steps(kind)
        print("  tree steps per member (one stream, cut %d): " % CUT
              + ", ".join("%d: %.1f" % (c, v[1] / v[0]) for c, v in sorted(st.items()))
              + "; all %.1f" % (sum(v[1] for v in st.values()) / sum(v[0] for v in st.values())))
        long_steps = sum(v[1] for c, v in st.items() if c >= 256)
        print("  steps in buckets >= 256: %.1f%% of the stream's steps" % (100.0 * long_steps / sum(v[1] for v in st.values())))


if __name__ == "__main__":
    main()
