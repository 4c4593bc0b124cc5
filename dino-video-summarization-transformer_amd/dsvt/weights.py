"""Storage-dtype views of nn.Parameters for the kernels.

bf16 mode: each weight is cast ONCE by the dsvt cast kernel and cached until the parameter
changes (tracked by its autograd version counter + storage pointer, so optimizer steps,
EMA updates, load_state_dict and .to() all invalidate it).  fp32 mode: the parameter
itself (no copy).

Stream safety: a cached copy is produced on whatever stream was current at the cache miss.
Every entry records an event after its producer; the first use from any OTHER stream waits on
that event (once per stream).  Callers that fan work out over side streams (MultiCropWrapper,
dino_forward) additionally call `prepare()` on the launching stream first, so all copies exist
before the side streams fork from it."""
import torch

from . import ops
from ._lib import DsvtError


class WeightCache:
    def __init__(self):
        self._c = {}
        self._tables = {}          # multi-tensor pointer / chunk tables of refresh(), by (src, dst) list

    @staticmethod
    def _sync(ent):
        """Order the current stream after the entry's producer (no-op on the producing stream)."""
        ev, waited = ent[-2], ent[-1]
        if ev is None:
            return
        cur = torch.cuda.current_stream()
        if cur.cuda_stream in waited:
            return
        if torch.cuda.is_current_stream_capturing():
            # cross-capture waits are illegal; a copy made before the capture must be finished
            if not ev.query():
                raise DsvtError("weight cache entry still in flight at HIP-graph capture: run one eager "
                                "forward (and synchronize) before capturing")
        else:
            cur.wait_event(ev)
        waited[cur.cuda_stream] = cur      # a reader: refresh() orders its in-place rewrite after it

    @staticmethod
    def _event():
        """(event after the producer, {stream id: stream} of the streams that use the entry)."""
        if torch.cuda.is_current_stream_capturing():
            return None, {}
        ev = torch.cuda.Event()
        ev.record()
        cur = torch.cuda.current_stream()
        return ev, {cur.cuda_stream: cur}

    @staticmethod
    def _after_readers(ents):
        """Order the current stream after everything queued so far on every OTHER stream that
        has read one of `ents` (the write-after-read hazard of an in-place rewrite): one event
        per such stream, recorded at its current tail."""
        cur = torch.cuda.current_stream()
        seen = {cur.cuda_stream}
        for ent in ents:
            for sid, s in ent[-1].items():
                if sid not in seen:
                    seen.add(sid)
                    ev = torch.cuda.Event()
                    ev.record(s)
                    cur.wait_event(ev)

    def getter(self, mode):
        def get(p, flat=False):
            t = p.detach()
            if flat:
                t = t.reshape(t.shape[0], -1)
            if t.dtype != torch.float32:
                raise TypeError("dsvt expects fp32 master parameters, got %s" % t.dtype)
            if mode == torch.float32:
                return t.contiguous()
            key = (id(p), flat)
            ent = self._c.get(key)
            if ent is not None and ent[0] == p._version and ent[1] == p.data_ptr():
                self._sync(ent)
                return ent[2]
            out = torch.empty(t.shape, device=t.device, dtype=mode)
            ops.cast(t.contiguous(), out)
            self._c[key] = (p._version, p.data_ptr(), out) + self._event()
            return out
        return get

    def padded(self, mode):
        """W [N, K] as [N, ldk] in the storage dtype with zero columns K..ldk-1 (ldk = K rounded
        up to 32 elements: one K step of the bf16 persistent GEMM / the fp32 MFMA K tile), cached
        like the casts.  Returns (w, ldk)."""
        def get(p, flat=False):
            t = p.detach()
            if flat:
                t = t.reshape(t.shape[0], -1)
            K = t.shape[1]
            q = 32
            ldk = (K + q - 1) // q * q
            key = (id(p), "pad", mode, flat)
            ent = self._c.get(key)
            if ent is not None and ent[0] == p._version and ent[1] == p.data_ptr():
                self._sync(ent)
                return ent[2], ldk
            out = torch.empty(t.shape[0], ldk, device=t.device, dtype=mode)
            ops.cast_pad(t.float().contiguous(), out)
            self._c[key] = (p._version, p.data_ptr(), out) + self._event()
            return out, ldk
        return get

    def padded_transposed(self, mode):
        """W^T [K, N] as [K, ldn] in the storage dtype with zero columns N..ldn-1 (ldn = N rounded up
        to the MFMA K tile): the B operand of an input-gradient GEMM dX = dY . W whose dY width N
        needs padding (the Video Swin C = 96 stage, train_ssl.py --arch swin).  Returns (wt, ldn)."""
        def get(p):
            t = p.detach()
            N = t.shape[0]
            q = 32
            ldn = (N + q - 1) // q * q
            key = (id(p), "padT", mode)
            ent = self._c.get(key)
            if ent is not None and ent[0] == p._version and ent[1] == p.data_ptr():
                self._sync(ent)
                return ent[2], ldn
            out = torch.empty(t.shape[1], ldn, device=t.device, dtype=mode)
            ops.cast_pad(t.t().contiguous().float(), out)
            self._c[key] = (p._version, p.data_ptr(), out) + self._event()
            return out, ldn
        return get

    def transposed(self, mode):
        """W^T [in, out] in the storage dtype (dsvt cast-transpose kernel), cached like the
        casts: the B operand of the backward's input-gradient GEMMs dX = dY . W."""
        def get(p):
            t = p.detach()
            if t.dtype != torch.float32 or t.dim() != 2:
                raise TypeError("dsvt expects 2-D fp32 master weights, got %s %s" % (t.dtype, tuple(t.shape)))
            key = (id(p), "T", mode)
            ent = self._c.get(key)
            if ent is not None and ent[0] == p._version and ent[1] == p.data_ptr():
                self._sync(ent)
                return ent[2]
            out = torch.empty(t.shape[1], t.shape[0], device=t.device, dtype=mode)
            ops.cast_transpose(t.contiguous(), out)
            self._c[key] = (p._version, p.data_ptr(), out) + self._event()
            return out
        return get

    def folded(self, mode, outer, inner):
        """outer(inner(x)) for two nn.Linear with nothing between them, as ONE Linear:
        W = Wo.Wi, b = Wo.bi + bo, formed in fp32 on the dsvt GEMM (then cast to `mode`) and
        cached until any of the four parameters changes.  Used for the temporal branch
        proj -> temporal_fc of the divided block (timesformer.py:83, 133-135: dropout 0)."""
        params = (outer.weight, outer.bias, inner.weight, inner.bias)
        stamp = tuple((p._version, p.data_ptr()) for p in params)
        key = ("fold", id(outer), id(inner), mode)
        ent = self._c.get(key)
        if ent is not None and ent[0] == stamp:
            self._sync(ent)
            return ent[1]
        wo, bo, wi, bi = (p.detach().float().contiguous() for p in params)
        dev = wo.device
        wi_t = wi.t().contiguous()                       # [in_i, out_i]: the GEMM's W[n][k] = Wi[k][n]
        w32 = torch.empty(wo.shape[0], wi.shape[1], device=dev, dtype=torch.float32)
        ops.gemm(wo, wi_t, None, w32)                    # W[m][n] = sum_k Wo[m][k] Wi[k][n]
        b32 = torch.empty(1, wo.shape[0], device=dev, dtype=torch.float32)
        ops.gemm(bi.reshape(1, -1), wo, bo, b32)         # b[n] = sum_k bi[k] Wo[n][k] + bo[n]
        b32 = b32.reshape(-1)
        if mode == torch.float32:
            w = w32
        else:
            w = torch.empty(w32.shape, device=dev, dtype=mode)
            ops.cast(w32, w)
        self._c[key] = (stamp, (w, b32)) + self._event()
        return w, b32

    def folded_t(self, mode, outer, inner):
        """(Wo.Wi)^T [in_i, out_o] in `mode`: the B operand of dX_inner_input = dY_outer . Wo . Wi
        (the backward of two nn.Linear with nothing between them in ONE GEMM), formed in fp32 and
        cast-transposed, cached until either weight changes."""
        params = (outer.weight, inner.weight)
        stamp = tuple((p._version, p.data_ptr()) for p in params)
        key = ("fold_t", id(outer), id(inner), mode)
        ent = self._c.get(key)
        if ent is not None and ent[0] == stamp:
            self._sync(ent)
            return ent[1]
        wo, wi = (p.detach().float().contiguous() for p in params)
        w32 = torch.empty(wo.shape[0], wi.shape[1], device=wo.device, dtype=torch.float32)
        ops.gemm(wo, wi.t().contiguous(), None, w32)     # W[m][n] = sum_k Wo[m][k] Wi[k][n]
        out = torch.empty(wi.shape[1], wo.shape[0], device=wo.device, dtype=mode)
        ops.cast_transpose(w32, out)
        self._c[key] = (stamp, out) + self._event()
        return out

    def ln_folded(self, linear, ln, heads=0):
        """(Wf, wsum, bias_f) of nn.Linear `linear` after nn.LayerNorm `ln` for the LayerNorm-folded
        GEMM (dsvt_gemm_lnx_fwd): Wf = bf16(W * gamma), wsum = its row sums, bias_f = b + W . beta,
        one dsvt_ln_fold_weights launch, cached until any of the four parameters changes.
        heads > 0: an attention qkv weight with its rows head-interleaved (dsvt_ln_fold_qkv_heads,
        the temporal-attention GEMM's order)."""
        params = (linear.weight, linear.bias, ln.weight, ln.bias)
        stamp = tuple((None, 0) if p is None else (p._version, p.data_ptr()) for p in params)
        key = ("lnfold", id(linear), id(ln), heads)
        ent = self._c.get(key)
        if ent is not None and ent[0] == stamp:
            self._sync(ent)
            return ent[1]
        W = linear.weight.detach()
        if W.dtype != torch.float32 or not W.is_contiguous():
            raise TypeError("dsvt expects contiguous fp32 master weights, got %s" % W.dtype)
        N, K = W.shape
        dev = W.device
        Wf = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        wsum = torch.empty(N, device=dev, dtype=torch.float32)
        bf = torch.empty(N, device=dev, dtype=torch.float32)
        b = None if linear.bias is None else linear.bias.detach()
        if heads:
            ops.ln_fold_qkv_heads(W, ln, b, Wf, wsum, bf, heads)
        else:
            ops.ln_fold_weights(W, ln, b, Wf, wsum, bf)
        self._c[key] = (stamp, (Wf, wsum, bf)) + self._event()
        return Wf, wsum, bf

    def refresh(self, params, mode, transposed=False, flat=()):
        """Bring the storage-dtype copies (transposed: the W^T copies) of many parameters up to
        date in ONE multi-tensor launch instead of one cast per weight -- after every optimizer
        / EMA step all of a model's copies are stale at once.  `flat`: ids of parameters used
        flattened to [rows, -1] (the patch-embedding conv).  Stale copies are rewritten in
        place, after every other stream that has read them (`_after_readers`); under HIP-graph
        capture (no cross-stream ordering to the past) they get fresh buffers instead."""
        if mode == torch.float32 or not params:
            return
        capturing = torch.cuda.is_current_stream_capturing()
        stale, reused = [], []
        for p in params:
            fl = id(p) in flat
            key = (id(p), "T", mode) if transposed else (id(p), fl)
            ent = self._c.get(key)
            if ent is not None and ent[0] == p._version and ent[1] == p.data_ptr():
                continue
            t = p.detach()
            if fl:
                t = t.reshape(t.shape[0], -1)
            if t.dtype != torch.float32 or not t.is_contiguous() or (transposed and t.dim() != 2):
                raise TypeError("dsvt expects contiguous fp32 master weights, got %s %s" % (t.dtype, tuple(t.shape)))
            shape = (t.shape[1], t.shape[0]) if transposed else tuple(t.shape)
            if (not capturing and ent is not None and tuple(ent[2].shape) == shape and ent[2].dtype == mode):
                out = ent[2]
                reused.append(ent)
            else:
                out = torch.empty(shape, device=t.device, dtype=mode)
            stale.append((key, p, t, out))
        if not stale:
            return
        self._after_readers(reused)
        from ._lib import call
        tkey = (transposed,) + tuple((t.data_ptr(), o.data_ptr(), tuple(t.shape)) for _, _, t, o in stale)
        tables = self._tables.get(tkey)
        dev = stale[0][2].device
        if tables is None:
            from .training import dev_table
            src = dev_table([t.data_ptr() for _, _, t, _ in stale], torch.int64, dev)
            dst = dev_table([o.data_ptr() for _, _, _, o in stale], torch.int64, dev)
            if transposed:
                rows = [t.shape[0] for _, _, t, _ in stale]
                cols = [t.shape[1] for _, _, t, _ in stale]
                tt, rc = [], []
                for i, (r, c) in enumerate(zip(rows, cols)):
                    for a in range((r + 63) // 64):
                        for b in range((c + 63) // 64):
                            tt.append(i)
                            rc.append((a << 16) | b)
                tables = (src, dst, dev_table(rows, torch.int64, dev), dev_table(cols, torch.int64, dev),
                          dev_table(tt, torch.int32, dev), dev_table(rc, torch.int32, dev), len(tt))
            else:
                from .training import TensorList
                tl = TensorList([t for _, _, t, _ in stale], dev)
                tables = (src, dst, tl.sizes, tl.ctensor, tl.cstart, tl.nchunks)
            if len(self._tables) > 16:
                self._tables.pop(next(iter(self._tables)))
            self._tables[tkey] = tables
        if transposed:
            src, dst, rows, cols, tt, rc, n = tables
            call("dsvt_cast_transpose_multi", src.data_ptr(), dst.data_ptr(), rows.data_ptr(), cols.data_ptr(),
                 tt.data_ptr(), rc.data_ptr(), n, ops._stream())
        else:
            src, dst, sizes, ct, cs, n = tables
            call("dsvt_cast_multi", src.data_ptr(), dst.data_ptr(), sizes.data_ptr(), ct.data_ptr(), cs.data_ptr(),
                 n, ops._stream())
        ev = self._event()
        for key, p, _, out in stale:
            self._c[key] = (p._version, p.data_ptr(), out) + ev

    def clear(self):
        self._c.clear()
        self._tables.clear()
