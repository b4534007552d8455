"""DistSampler's particle / score exchange on torch.distributed.

On MI355X the process group is `nccl` (= RCCL over xGMI) and every buffer is
a device tensor, so the collectives run stream-ordered on the GPU.  The same
functions accept a `gloo` group (CPU rehearsal / tests); gloo is given host
copies.  Reference call sites: dist.isend/irecv (dsvgd/distsampler.py:136,143),
dist.all_gather (:156), dist.all_reduce SUM (:170).
"""
import torch
import torch.distributed as dist


def _is_gloo(group=None):
    return dist.get_backend(group) == "gloo"


def all_gather_blocks(own, out, group=None):
    """out (S*m, d) <- concat over ranks of `own` (m, d)   [distsampler.py:152-158]."""
    if own.is_cuda and not _is_gloo(group):
        dist.all_gather_into_tensor(out, own.contiguous(), group=group)
        return
    src = own.detach().cpu().contiguous()
    parts = [torch.empty_like(src) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, src, group=group)
    out.copy_(torch.cat(parts).to(out.device))


def all_gather_in_place(full, start, end, group=None):
    """full[start:end] is this rank's block at rank * (end - start): gather the
    other blocks around it in place (RCCL in-place all-gather, no staging
    copy).  Returns False (nothing done) where that layout or backend does not
    hold; the caller then uses all_gather_blocks."""
    if not (full.is_cuda and full.is_contiguous()) or _is_gloo(group):
        return False
    m = end - start
    if m <= 0 or start != dist.get_rank(group) * m or full.shape[0] != m * dist.get_world_size(group):
        return False
    dist.all_gather_into_tensor(full, full[start:end], group=group)
    return True


def all_reduce_sum(t, group=None):
    """In-place SUM over ranks   [distsampler.py:170]."""
    if t.is_cuda and not _is_gloo(group):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return
    h = t.detach().cpu()
    dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    t.copy_(h.to(t.device))


def all_reduce_max(t, group=None):
    """In-place MAX over ranks (device tensors on RCCL, host staging on
    gloo); returns t."""
    if t.is_cuda and not _is_gloo(group):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return t
    h = t.detach().cpu()
    dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
    t.copy_(h.to(t.device))
    return t


def ring_shift(send, recv, rank, size, group=None):
    """send -> rank+1, recv <- rank-1   [distsampler.py:131-150].

    `rank` and `size` are the caller's shard rank and count inside `group`
    (group-local ranks, the order all_gather uses); the peers are addressed
    as group ranks (`group_peer`), so a subgroup of a larger world sends to
    the right processes."""
    dst, src = (rank + 1) % size, (rank - 1 + size) % size
    exchange_p2p([(send, dst)], [(recv, src)], group)


def exchange_p2p_async(sends, recvs, group=None):
    """exchange_p2p without the join: returns a callable that joins the
    transfers.  On RCCL the ops are posted on the process group's stream
    (after the work already queued on the current stream) and the join makes
    the current stream wait for them, so kernels enqueued in between overlap
    the transfers; gloo completes them here (host staging) and returns a no-op."""
    dev = any(t.is_cuda for t, _ in list(sends) + list(recvs))
    if not (dev and not _is_gloo(group)) or (not sends and not recvs):
        exchange_p2p(sends, recvs, group)
        return lambda: None
    ops = [dist.P2POp(dist.isend, t, group=group, group_peer=p) for t, p in sends]
    ops += [dist.P2POp(dist.irecv, t, group=group, group_peer=p) for t, p in recvs]
    works = dist.batch_isend_irecv(ops)

    def join():
        for w in works:
            w.wait()
    return join


def probe_p2p(send_peers, recv_peers, rank, device, group=None, _corrupt=False):
    """Route check of a point-to-point plan on the live backend, through the
    same path the step uses (exchange_p2p_async: post, kernels on the
    current stream, join, read on the current stream): every rank sends each
    planned peer a small tensor tagged (sender, receiver), produced by a
    kernel right before the post, and checks what arrives from each planned
    source.  The verdicts are combined over the group (MIN), so every rank
    gets the same answer -- DistSampler falls back to the row-block layout on
    all ranks together when any rank saw a wrong or missing message.
    `_corrupt` (tests only) spoils this rank's first received buffer."""
    L = 259
    ramp = torch.arange(L, dtype=torch.float32, device=device)

    def tag(src, dst):
        return float(src * 8192 + dst + 1)
    sb = [torch.empty(L, device=device) for _ in send_peers]
    rb = [torch.full((L,), float("nan"), device=device) for _ in recv_peers]
    for t, p in zip(sb, send_peers):
        torch.add(ramp, tag(rank, p), out=t)
    join = exchange_p2p_async(list(zip(sb, send_peers)), list(zip(rb, recv_peers)), group)
    busy = torch.ones(256, 256, device=device)
    for _ in range(3):                     # work queued between the post and the join
        busy = torch.mm(busy, busy) * (1.0 / 256)
    join()
    if _corrupt and rb:
        rb[0][0] += 1.0            # a wrong payload: the comparison below must catch it
    ok = True
    for t, p in zip(rb, recv_peers):
        ok = ok and bool(torch.equal(t, ramp + tag(p, rank)))
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64,
                        device=device if not _is_gloo(group) else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item() == 1)


def exchange_p2p(sends, recvs, group=None):
    """Point-to-point transfers in one batch: sends = [(tensor, group_rank)],
    recvs = [(tensor, group_rank)], peers as ranks of `group`.  On RCCL the
    ops are posted together (batch_isend_irecv: one fused group call, each
    pair of peers on its own xGMI link) and joined before returning; on gloo
    the tensors are staged through host copies."""
    if not sends and not recvs:
        return
    dev = any(t.is_cuda for t, _ in list(sends) + list(recvs))
    if dev and not _is_gloo(group):
        ops = [dist.P2POp(dist.isend, t.contiguous(), group=group, group_peer=p) for t, p in sends]
        ops += [dist.P2POp(dist.irecv, t, group=group, group_peer=p) for t, p in recvs]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        return
    work, host = [], []
    for t, p in sends:
        work.append(dist.isend(t.detach().cpu().contiguous(), group=group, group_dst=p))
    for t, p in recvs:
        h = torch.empty(t.shape, dtype=t.dtype)
        host.append((t, h))
        work.append(dist.irecv(h, group=group, group_src=p))
    for w in work:
        w.wait()
    for t, h in host:
        t.copy_(h.to(t.device))
