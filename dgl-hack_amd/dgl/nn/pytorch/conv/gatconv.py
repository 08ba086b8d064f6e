"""GATConv (``python/dgl/nn/pytorch/conv/gatconv.py:13-171``).

Same parameters, initialisation and math as the reference: projection
(torch GEMM), el / er attention terms, ``u_add_v`` SDDMM, LeakyReLU,
max-stabilised ``edge_softmax`` and ``u_mul_e_sum`` with the attention
broadcast over the head dimension (the load-balanced HIP kernel).  When the
head size suits the fused kernel, the middle of that chain (u_add_v ..
u_mul_e_sum) runs as ONE fused HIP kernel (``dgl.backend.fused_gat``; same math,
max-stabilised in both forms), attention dropout in training included: by default
the module's own ``nn.Dropout`` draws over an (E, H, 1) tensor in edge-id order -- the
draws the reference's ``self.attn_drop(edge_softmax(...))`` (gatconv.py:154) makes under
the same seed -- recomputed inside the fused kernels from the generator state
(``dgl.kernel.dropout_draw``; once checked against torch.native_dropout per device), or
drawn by torch.native_dropout and packed to one keep word per edge
(``attn_drop_mask = "module"``); ``attn_drop_mask =
"hashed"`` opts into a mask hashed inside the kernels from a per-call seed (the same
Bernoulli(1 - p) per edge and head, not torch's draws; no (E, H) tensors).  Set
``use_fused = False`` on the module to force the unfused composition.
The reference's unconditional ``th.cuda.synchronize()`` + timing prints
(:146-170) are not reproduced.
"""
import numpy as np
import torch as th
from torch import nn

from .... import backend as B
from .... import function as fn
from .... import kernel as K
from ..softmax import edge_softmax
from ..softmax import _apply as _edge_softmax_on
from ..softmax import _apply_leaky as _leaky_edge_softmax_on
from ..softmax import _apply_node_logits as _node_logit_edge_softmax_on

# run the unfused composition in in-CSR position order (GATConv._position_space);
# False: edge-id order throughout, as the reference
POSITION_SPACE = True
# the composition's leaky_relu -> edge_softmax pair as one fused softmax call (False: two)
FUSED_LEAKY = True
# the position-space composition's backward as ONE fused pass pair (backend.GatComposition:
# the forward unchanged, the gradients within fp32 rounding); False: step by step
FUSED_COMPOSITION_BACKWARD = True
# the fused route's module-mask draw: torch.native_dropout -- what nn.Dropout's forward
# runs on a ROCm tensor with 0 < p < 1 -- on an UNINITIALISED (E, H, 1) tensor of this
# dtype, keeping only its boolean mask: the draws depend on the generator, the element
# count and the vector width, not on the values (scripts/dropout_draw_probe.py)
MODULE_DRAW_DTYPE = th.float32
# ... or, when dgl.kernel.dropout_draw_ok (checked once per device against torch itself),
# those draws recomputed inside the fused walks from the generator state (no mask, no
# gathers; DGLMIFusedGatDraw*)
MODULE_DRAW_IN_KERNEL = True
# el / er (gatconv.py:137-138) as one pass over the features each way on every route
# (dgl.backend.attn_logits: torch's bits -- the same pairwise summation order -- so the
# composition's forward keeps the reference's bits; the gradients within fp32 rounding)
FUSED_ATTN_LOGITS = True


def expand_as_pair(x):
    return x if isinstance(x, tuple) else (x, x)


class Identity(nn.Module):
    def forward(self, x):
        return x


class GATConv(nn.Module):
    def __init__(self, in_feats, out_feats, num_heads, feat_drop=0., attn_drop=0.,
                 negative_slope=0.2, residual=False, activation=None):
        super(GATConv, self).__init__()
        self._num_heads = num_heads
        self._in_src_feats, self._in_dst_feats = expand_as_pair(in_feats)
        self._out_feats = out_feats
        if isinstance(in_feats, tuple):
            self.fc_src = nn.Linear(self._in_src_feats, out_feats * num_heads, bias=False)
            self.fc_dst = nn.Linear(self._in_dst_feats, out_feats * num_heads, bias=False)
        else:
            self.fc = nn.Linear(self._in_src_feats, out_feats * num_heads, bias=False)
        self.attn_l = nn.Parameter(th.FloatTensor(size=(1, num_heads, out_feats)))
        self.attn_r = nn.Parameter(th.FloatTensor(size=(1, num_heads, out_feats)))
        self.feat_drop = nn.Dropout(feat_drop)
        self.attn_drop = nn.Dropout(attn_drop)
        self.leaky_relu = nn.LeakyReLU(negative_slope)
        if residual:
            if self._in_dst_feats != out_feats:
                self.res_fc = nn.Linear(self._in_dst_feats, num_heads * out_feats, bias=False)
            else:
                self.res_fc = Identity()
        else:
            self.register_buffer("res_fc", None)
        self.reset_parameters()
        self.activation = activation
        self.negative_slope = negative_slope
        self.use_fused = True
        # "module": attention dropout with this module's nn.Dropout draws (the
        # reference's); "hashed": the fused kernels' own hashed mask (faster, other draws)
        self.attn_drop_mask = "module"

    # FusedGATConv builds attn_drop but never applies it (fusedGatConv.py:80,152)
    _applies_attn_drop = True

    def _attn_drop_active(self):
        return self._applies_attn_drop and self.training and self.attn_drop.p > 0

    def _fused_ok(self):
        # attention dropout in training runs inside the fused kernels (dgl.backend.fused_gat)
        if not self.use_fused:
            return False
        return self._fused_dim() is not None

    def _fused_route(self, graph, n_rows):
        """Whether this call takes the fused kernels: the head size suits them, the
        graph has 32-bit device indices (a 2^31+-edge graph takes the composition,
        whose kernels have 64-bit offsets) and, with attention dropout in training,
        the gathered tables stay below 2^31 elements and there are at most 32 heads (the
        dropout walks are built with 32-bit offsets and stage 32 keep bits per edge;
        ``capi.cpp`` gat_set_dropout).  ``graph``: a DGLGraph or
        an ImmutableGraphIndex; ``n_rows``: the larger of its source / destination
        row counts."""
        if not self._fused_ok():
            return False
        if hasattr(graph, "in_csr"):  # an ImmutableGraphIndex: its device CSRs
            if graph.in_csr.bits != 32:
                return False
        elif getattr(graph._graph, "device_bits", lambda: 32)() != 32:
            return False
        if self._attn_drop_active():
            if self.attn_drop.p >= 1.0:
                return False  # nn.Dropout(1) zeroes every weight: the composition
            if self.attn_drop_mask == "module":
                # the module's draws: a plain nn.Dropout (scale 1 / (1 - p)) over the
                # graph's own edge ids (keep words indexed by edge id)
                if type(self.attn_drop) is not nn.Dropout or self.attn_drop.inplace:
                    return False
                gidx = graph if hasattr(graph, "in_csr") else \
                    graph._graph.get_immutable_gidx(self.attn_l.device)
                if not gidx.eid_perm:
                    return False
            elif self.attn_drop_mask != "hashed":
                raise ValueError("attn_drop_mask must be 'module' or 'hashed'")
            # the dropout walks stage <= 32 keep bits per edge (capi.cpp gat_set_dropout)
            return (self._num_heads <= 32
                    and n_rows * self._num_heads * self._fused_dim() < (1 << 31))
        return True

    def _position_space(self, graph, feat_src):
        """Whether the composition may run with edge ids = in-CSR positions: the logits
        and attention are internal to this call (the reference sets them on a
        ``local_var`` graph), so they can live in the walk's order instead of edge-id
        order -- every per-edge read and write streams instead of landing on a random
        line per edge.  Whole graphs only (edge ids a permutation).  Attention dropout
        in training keeps ``nn.Dropout``'s draws in edge-id order (the reference's
        composition): the module draws a mask of ones in edge-id order, gathered into
        walk order (``_composed_in_positions``); another dropout module keeps the
        edge-id composition."""
        if not POSITION_SPACE or not feat_src.is_cuda:
            return False
        if self._attn_drop_active() and \
                (type(self.attn_drop) is not nn.Dropout or self.attn_drop.inplace):
            return False
        if not hasattr(getattr(graph, "_graph", None), "get_immutable_gidx"):
            return False
        gidx = graph._graph.get_immutable_gidx(feat_src.device)
        return gidx.eid_perm and gidx.in_csr.nnz > 0

    def _composed_in_positions(self, graph, feat_src, el, er):
        """u_add_v, LeakyReLU, edge_softmax and u_mul_e_sum -- the reference's
        composition, the same kernels -- on the graph's in-CSR position view
        (ImmutableGraphIndex.position_view): the same values summed in the same order,
        bit-identical to the edge-id composition (tests/test_nn_gpu.py)."""
        gidx = graph._graph.get_immutable_gidx(feat_src.device)
        view = gidx.position_view("in")
        n_dst, m = view.num_dst, view.number_of_edges()
        if (FUSED_COMPOSITION_BACKWARD and FUSED_LEAKY and type(self.leaky_relu) is nn.LeakyReLU
                and B.gat_composition_ok(gidx, feat_src, el, er)):
            # the same forward; the backward as the fused GAT's walks (GatComposition) --
            # with attention dropout when its draws can be recomputed in the walks
            draw = None
            if self._attn_drop_active():
                p = float(self.attn_drop.p)
                numel = m * self._num_heads
                if (MODULE_DRAW_IN_KERNEL and 0.0 < p < 1.0 and self._num_heads <= 32 and numel > 0
                        and K.dropout_draw_ok(feat_src.device)):
                    draw = K.dropout_draw(feat_src.device, numel, p)
            if draw is not None:
                return B.gat_composition(gidx, view, feat_src, el, er, self.leaky_relu.negative_slope,
                                         draw=draw)
            if not self._attn_drop_active():
                return B.gat_composition(gidx, view, feat_src, el, er, self.leaky_relu.negative_slope)
        if type(self.leaky_relu) is nn.LeakyReLU and FUSED_LEAKY:
            # u_add_v and the activation inside the softmax's passes: the logits are
            # computed where they are read, never stored (bit-identical to the three steps)
            a = _node_logit_edge_softmax_on(view, el, er, n_dst, self.leaky_relu.negative_slope)
        else:
            e = B.binary_reduce("none", "add", view, B.SRC, B.DST, el, er, m)
            a = _edge_softmax_on(view, self.leaky_relu(e), n_dst)
        if self._attn_drop_active():
            # nn.Dropout's draws in edge-id order, as dropout(a) in the edge-id
            # composition: (1 * keep) * scale per edge, gathered into walk order; a times
            # it is dropout's (a * keep) * scale bit for bit, and so is the gradient.
            # With the draws recomputable (dgl.kernel.dropout_draw_ok) the walk-order
            # scale is written directly from them (no ones, no (E, H) draw, no gather).
            numel = m * self._num_heads
            p = float(self.attn_drop.p)
            if (MODULE_DRAW_IN_KERNEL and 0.0 < p < 1.0 and self._num_heads <= 32 and numel > 0
                    and K.dropout_draw_ok(a.device)):
                scale = K.dropout_draw_scale(K.dropout_draw(a.device, numel, p), self._num_heads,
                                             gidx.in_csr.data, m, a.device)
                a = a * scale.view(a.shape)
            else:
                scale = self.attn_drop(a.new_ones(a.shape))
                a = a * K.gather_rows(scale, gidx.in_csr.data)
        return B.binary_reduce("sum", "mul", view, B.SRC, B.EDGE, feat_src, a, n_dst)

    def _fused_dim(self):
        """Head width for the fused kernel (the output width itself, or padded to
        the next supported one; see dgl.kernel.fused_gat_head_dim)."""
        if not hasattr(self, "_fdim"):
            self._fdim = K.fused_gat_head_dim(self._num_heads, self._out_feats)
        return self._fdim

    def _fused(self, graph, feat_src, el, er):
        d = self._fused_dim()
        kw = {}
        if self._attn_drop_active():
            p = float(self.attn_drop.p)
            if self.attn_drop_mask == "hashed":
                kw = {"attn_drop": p}
            else:
                # this module's nn.Dropout draws on (E, H, 1) in edge-id order: the RNG
                # draws of the reference's attn_drop(a) (same shape, same layout), packed
                # from the dropout's boolean mask to one keep word per edge; kept weights
                # take torch's scale float(1 / float(1 - p)) (its fused dropout kernel's)
                gidx = graph if hasattr(graph, "in_csr") else \
                    graph._graph.get_immutable_gidx(feat_src.device)
                numel = gidx.in_csr.nnz * self._num_heads
                if MODULE_DRAW_IN_KERNEL and numel > 0 and K.dropout_draw_ok(feat_src.device):
                    # the same draws recomputed inside the walks: the generator advances
                    # as this module's nn.Dropout would, no mask is materialised
                    kw = {"draw": K.dropout_draw(feat_src.device, numel, p)}
                    return self._fused_call(graph, feat_src, el, er, d, kw)
                draw = th.empty((gidx.in_csr.nnz, self._num_heads, 1), device=feat_src.device,
                                dtype=MODULE_DRAW_DTYPE)
                _, keep = th.native_dropout(draw, p, True)
                del draw
                kw = {"keep": K.gat_keep_bits(keep),
                      "keep_scale": float(np.float32(1.0 / float(np.float32(1.0 - p))))}
                del keep
        return self._fused_call(graph, feat_src, el, er, d, kw)

    def _fused_call(self, graph, feat_src, el, er, d, kw):
        if d == self._out_feats:
            return B.fused_gat(graph, feat_src, el, er, self.negative_slope, **kw)
        ft = th.nn.functional.pad(feat_src, (0, d - self._out_feats))
        return B.fused_gat(graph, ft, el, er, self.negative_slope, **kw)[..., :self._out_feats]

    def reset_parameters(self):
        gain = nn.init.calculate_gain("relu")
        if hasattr(self, "fc"):
            nn.init.xavier_normal_(self.fc.weight, gain=gain)
        else:
            nn.init.xavier_normal_(self.fc_src.weight, gain=gain)
            nn.init.xavier_normal_(self.fc_dst.weight, gain=gain)
        nn.init.xavier_normal_(self.attn_l, gain=gain)
        nn.init.xavier_normal_(self.attn_r, gain=gain)
        if isinstance(self.res_fc, nn.Linear):
            nn.init.xavier_normal_(self.res_fc.weight, gain=gain)

    def forward(self, graph, feat):
        graph = graph.local_var()
        if isinstance(feat, tuple):
            h_src = self.feat_drop(feat[0])
            h_dst = self.feat_drop(feat[1])
            feat_src = B.project(h_src, self.fc_src.weight.t()).view(-1, self._num_heads, self._out_feats)
            feat_dst = B.project(h_dst, self.fc_dst.weight.t()).view(-1, self._num_heads, self._out_feats)
        else:
            h_src = h_dst = self.feat_drop(feat)
            feat_src = feat_dst = B.project(h_src, self.fc.weight.t()).view(-1, self._num_heads, self._out_feats)
        fused = self._fused_route(graph, max(feat_src.shape[0], feat_dst.shape[0]))
        if FUSED_ATTN_LOGITS and K.attn_logits_ok(feat_src, feat_dst, self.attn_l, self.attn_r):
            el, er = B.attn_logits(feat_src, feat_dst, self.attn_l, self.attn_r)
        else:
            el = (feat_src * self.attn_l).sum(dim=-1).unsqueeze(-1)
            er = (feat_dst * self.attn_r).sum(dim=-1).unsqueeze(-1)
        if fused:
            rst = self._fused(graph, feat_src, el, er)
        elif not isinstance(feat, tuple) and self._position_space(graph, feat_src):
            rst = self._composed_in_positions(graph, feat_src, el, er)
        else:
            graph.srcdata.update({"ft": feat_src, "el": el})
            graph.dstdata.update({"er": er})
            graph.apply_edges(fn.u_add_v("el", "er", "e"))
            e = graph.edata.pop("e")
            if type(self.leaky_relu) is nn.LeakyReLU and FUSED_LEAKY and e.is_cuda and \
                    hasattr(graph._graph, "get_immutable_gidx"):
                gidx = graph._graph.get_immutable_gidx(e.device)
                a = _leaky_edge_softmax_on(gidx, e, graph.number_of_nodes(),
                                           self.leaky_relu.negative_slope)
            else:
                a = edge_softmax(graph, self.leaky_relu(e))
            graph.edata["a"] = self.attn_drop(a) if self._applies_attn_drop else a
            graph.update_all(fn.u_mul_e("ft", "a", "m"), fn.sum("m", "ft"))
            rst = graph.dstdata["ft"]
        if self.res_fc is not None:
            resval = self.res_fc(h_dst).view(h_dst.shape[0], -1, self._out_feats)
            rst = rst + resval
        if self.activation:
            rst = self.activation(rst)
        return rst
