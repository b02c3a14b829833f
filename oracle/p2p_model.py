"""Oracle (test infrastructure only): MPI point-to-point matching model.

Only tests/ may import this module; the product (mpi.jl_amd/) never does.

Restates the matching rules MPICH 3.3.2 implements for MPI_Recv / MPI_Irecv
(the libmpi behind src/pointtopoint.jl:266-339): messages from one source are
non-overtaking (arrival order = send order per (source, destination) pair);
a receive names a source (or MPI_ANY_SOURCE) and a tag (or MPI_ANY_TAG);
when a receive is posted it takes the EARLIEST arrived, unmatched message
that matches; when a message arrives it goes to the EARLIEST posted,
unmatched receive that matches.  Pinned by the MPICH-recorded scenarios in
tests/golden/p2p_golden.json ("tag_order" covers both orders with a wildcard).
"""
from __future__ import annotations

ANY_SOURCE = -2
ANY_TAG = -1


def _match(rsrc, rtag, msrc, mtag):
    return (rsrc == ANY_SOURCE or rsrc == msrc) and (rtag == ANY_TAG or rtag == mtag)


def match_unexpected_first(arrived, recvs):
    """Every message has arrived before any receive is posted.

    arrived: list of (src, tag, msg_id) in arrival order (per-source order =
             send order; interleaving across sources only matters for
             ANY_SOURCE receives).
    recvs:   list of (src, tag) in post order.
    Returns the matched msg_id per receive (None if nothing matches).
    """
    taken = [False] * len(arrived)
    out = []
    for rsrc, rtag in recvs:
        got = None
        for i, (msrc, mtag, mid) in enumerate(arrived):
            if not taken[i] and _match(rsrc, rtag, msrc, mtag):
                taken[i] = True
                got = mid
                break
        out.append(got)
    return out


def match_posted_first(recvs, arrived):
    """Every receive is posted before any message arrives: each message, in
    arrival order, goes to the earliest posted receive it matches."""
    owner = [None] * len(recvs)
    for msrc, mtag, mid in arrived:
        for j, (rsrc, rtag) in enumerate(recvs):
            if owner[j] is None and _match(rsrc, rtag, msrc, mtag):
                owner[j] = mid
                break
    return owner
