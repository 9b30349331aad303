"""The hot-path carrier plugins on the SELFRec surface (``selfrec.py``), with the reference's
training loops (paths relative to /root/reference/HD_SELFRec):

* :class:`HCCF`     — model/graph/HCCF.py:26-133 (HCCFEncoder, BPR + per-layer InfoNCE);
* :class:`HGNN_HD4` — model/graph/HGNN_HD4.py:32-251 with ``--mode=local_only`` (the ED-HNN
  "hypergraph diffusion" LocalAwareEncoder; the reference's group / full modes are broken as
  shipped, SURVEY.md §0.5, and are rejected here);
* :class:`HGNN_HD3` — model/graph/HGNN_HD3.py:37-266, the same plugin around the SpMM-form
  ED-HNN encoder (``encoders.LocalAwareEncoderHD3``);
* :class:`HGCN`     — model/graph/HGCN.py:15-164 (HGCNConv stack with per-layer
  TransformerEncoder self-attention);
* :class:`HCCF_sharded` — HCCF's loop on user-row shards under torch.distributed (no reference
  counterpart: the north_star's multi-GPU partition carried up to the plugin);
* :class:`HGNN_HD4_sharded` — HGNN_HD4 local_only on user-row shards (configs[3]'s
  "hypergraph diffusion, user-row sharded");
* :class:`HCCF_diffusion` — model/graph/HCCF_diffusion.py:22-129 (HCCF's loop with the ED-HNN
  block on the learned hypergraph, ``encoders.HCCFDiffusionEncoder``);
* :class:`DHCF`     — model/graph/DHCF.py:19-185 (HGCNConv on the interaction matrix, which
  the reference densifies, for users and items).

Each keeps the reference's constructor, config keys, optimiser / scheduler settings, loss
arithmetic and evaluation cadence — including its quirks (HCCF clips gradients before
``backward`` and never resets its loss list; HGNN_HD4 steps its scheduler and switches to
``eval()`` inside the batch loop; HGCN keeps its transformer layers in a plain list, so they
are not trained) — so a run takes the same steps. What runs underneath is this build's: batches
from ``sampler.next_batch_pairwise`` (bit-identical to util/sampler.py), the encoders of
``encoders.py`` on libhgd, ``functional.contrast_loss`` for ``contrastLoss`` and the device
evaluation of ``GraphRecommender``.

Drop-edge masks come from torch's default CPU generator exactly as the reference draws them
(natively, ``layers.torch_cpu_keep_mask``), so runs are reproducible against the reference for a
seed. ``kwargs['hgd_device_rng'] = True`` draws them on the device instead (same Bernoulli
distribution, a different stream, no host work in the step).
"""
from __future__ import annotations

import os
import random
import time

import numpy as np
import torch
import torch.nn as nn
from torch.optim.lr_scheduler import ReduceLROnPlateau

from .optim import ReferenceAdam, calibrated_variant

from .encoders import (HCCFDiffusionEncoder, HCCFEncoder, LocalAwareEncoder,
                       LocalAwareEncoderHD3, sparse_tensor_of)
from .functional import (bpr_index_errors, bpr_loss_rows, contrast_loss, contrast_loss_layers,
                         split_rows, unique_long, unique_long_n, unique_long_n_group)
from .layers import HGCNConv, SpAdjDropEdge
from .sampler import next_batch_pairwise
from .selfrec import GraphRecommender, early_stopping


def bpr_loss(user_emb, pos_item_emb, neg_item_emb):
    """util/loss_torch.py:5-9."""
    pos_score = torch.mul(user_emb, pos_item_emb).sum(dim=1)
    neg_score = torch.mul(user_emb, neg_item_emb).sum(dim=1)
    return torch.mean(-torch.log(10e-6 + torch.sigmoid(pos_score - neg_score)))


def l2_reg_loss(reg, *args):
    """util/loss_torch.py:17-21."""
    emb_loss = 0
    for emb in args:
        emb_loss += torch.norm(emb, p=2)
    return emb_loss * reg


def _device_drop_edge(dropper, kwargs) -> None:
    """The drop-edge result of every step is a masked VIEW of the parent adjacency (no
    compaction, no kept-count or split-plan read), with the InfoNCE node counts kept on the
    device too (:meth:`HCCF.ssl_loss`): an eager step makes no host read. The masks stay the
    reference's CPU ``torch.rand`` stream (bit-identical drops), drawn natively ahead of the
    step into per-call slots. Yelp shape 1.93 ms per eager step against 2.9 ms with compacted
    children (``scripts/bench_hccf.py``); on a Zipf-skewed catalogue, whose compacted children
    re-plan their split rows every step, 2.9 against 4.8 ms (``scripts/profile_plugin_steps.py``).
    ``hgd_compact_drop`` keeps the compacted children (the reference's sparse tensors; the
    sums differ from the view's only in the order of split rows' partials). ``hgd_device_rng``:
    the masks come from a device seed counter instead (same Bernoulli(keep) per edge, a
    different stream, no host work)."""
    dropper.device_rng = bool(kwargs.get('hgd_device_rng', False))
    dropper.capture_safe = not bool(kwargs.get('hgd_compact_drop', False))


class HCCF(GraphRecommender):
    """model/graph/HCCF.py:26-133."""

    # the training loop replays its steps from a HIP graph unless hgd_graph=False (or the
    # compacted drop-edge children are asked for): bitwise the eager steps, ~1.3 vs ~1.9 ms per
    # Yelp-shaped step
    _graph_default = True

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        GraphRecommender.__init__(self, conf, training_set, test_set, knowledge_set, **kwargs)
        self.model = HCCFEncoder(kwargs, self.data, self.device)
        _device_drop_edge(self.model.edgeDropper, kwargs)
        self._parse_config(self.config, kwargs)
        self.model.to(self.device)
        self._init_optimizer(kwargs)

    def _init_optimizer(self, kwargs):
        # hgd_graph: the training step replayed from one HIP graph (graphs.CapturedStep) — the
        # drop-edge masks as views filled before each replay, device-side InfoNCE node counts.
        # The optimizer is the reference's torch.optim.Adam(lr=float) (HCCF.py:33): inside the
        # graph as optim.ReferenceAdam (one kernel, its per-step scalars refilled before each
        # replay; bitwise torch's Adam — calibrated on the device, optim.calibrated_variant), or,
        # if no kernel variant is bitwise torch's on this build, torch's own Adam stepping eagerly
        # after each replay. Replayed steps are bitwise the eager steps either way.
        # hgd_capturable_adam=True puts torch's capturable fused Adam in the graph instead (not
        # the reference's rounding of the bias corrections: scripts/diag/diag_adam_bitwise.py)
        default = self._graph_default and not kwargs.get('hgd_compact_drop', False)
        self.graph_mode = bool(kwargs.get('hgd_graph', default))
        self._captured = None
        self._adam_in_graph = self.graph_mode and bool(kwargs.get('hgd_capturable_adam', False))
        self._adam_kernel = False
        if self.graph_mode:
            # the drop-edge masks stay the reference's CPU torch.rand stream (drawn on the host
            # before each replay into the buffers the graph reads) unless hgd_device_rng asks
            # for device draws
            self.model.edgeDropper.device_rng = bool(kwargs.get('hgd_device_rng', False))
            self.model.edgeDropper.capture_safe = True
        if self._adam_in_graph:
            lr = torch.tensor(self.lRate, dtype=torch.float32, device=self.device)
            # fused: one multi-tensor kernel per step instead of the ~15 foreach passes
            self.optimizer = torch.optim.Adam(self.model.parameters(), lr=lr, capturable=True,
                                              fused=True)
        elif self.graph_mode and calibrated_variant(self.device) is not None:
            self.optimizer = ReferenceAdam(self.model.parameters(), lr=self.lRate)
            self._adam_in_graph = self._adam_kernel = True
        else:
            self.optimizer = torch.optim.Adam(self.model.parameters(), lr=self.lRate)
        self.scheduler = ReduceLROnPlateau(self.optimizer, 'min', factor=self.lr_decay,
                                           patience=5)

    def _parse_config(self, config, kwargs):  # HCCF.py:39-59
        self.maxEpoch = int(kwargs['max_epoch'])
        self.batchSize = int(kwargs['batch_size'])
        self.lRate = float(kwargs['lrate'])
        self.lr_decay = float(kwargs['lr_decay'])
        self.reg = float(kwargs['reg'])
        self.latent_size = int(kwargs['embedding_size'])
        self.drop_rate = float(kwargs['drop_rate'])
        self.leaky = float(kwargs['p'])
        self.nLayers = int(kwargs['n_layers'])
        self.ss_rate = float(kwargs['cl_rate'])
        self.hyperDim = int(config['hyper.size'])
        self.dropRate = float(config['dropout'])
        self.negSlove = float(config['leaky'])
        self.temp = float(config['temp'])
        self.seed = int(kwargs['seed'])
        self.early_stopping_steps = int(kwargs['early_stopping_steps'])

    def calcLosses(self, ancs, poss, negs, gcnEmbedsLst, hyperEmbedsLst, reg):  # :61-70
        return bpr_loss(ancs, poss, negs), HCCF.ssl_loss(self, ancs, poss, gcnEmbedsLst,
                                                          hyperEmbedsLst)

    def ssl_loss(self, ancs, poss, gcnEmbedsLst, hyperEmbedsLst):  # :62-67
        nu = self.data.n_users
        # torch.unique(ancs.long()) / torch.unique(poss.long()) are the same in every layer of the
        # reference's loop: computed once here (each is a device→host read — or, in graph mode
        # and with device drop-edge masks, capacity-sized with the count kept on the device)
        dropper = getattr(getattr(self, "model", None), "edgeDropper", None)
        if getattr(self, "graph_mode", False) or getattr(dropper, "capture_safe", False):
            (u_nodes, u_cnt), (p_nodes, p_cnt) = unique_long_n_group(
                [ancs, poss], [nu, self.data.n_items])  # both lists in one launch per kernel
        else:
            u_nodes, p_nodes = unique_long(ancs), unique_long(poss)
            u_cnt = p_cnt = None
        # every layer's user and item terms (embeds1 = gcnEmbedsLst[i].detach(), embeds2 =
        # hyperEmbedsLst[i]) as one op: one launch per kernel for the whole loop when the node
        # counts are on the device (functional.contrast_loss_layers)
        sslLoss = contrast_loss_layers([gcnEmbedsLst[i].detach() for i in range(self.nLayers)],
                                       [hyperEmbedsLst[i] for i in range(self.nLayers)], nu,
                                       u_nodes, p_nodes, self.temp, u_cnt, p_cnt)
        sslLoss *= self.ss_rate
        return sslLoss

    def train_step(self, user_idx, pos_idx, neg_idx) -> torch.Tensor:
        """One batch of HCCF.py:79-97; returns the (device) batch loss."""
        batch_loss = self.forward_backward(user_idx, pos_idx, neg_idx)
        self.optimizer.step()
        return batch_loss

    def forward_backward(self, user_idx, pos_idx, neg_idx) -> torch.Tensor:
        """:meth:`train_step` up to the optimizer step (HCCF.py:79-95): the parameters' .grad
        hold the batch's gradients afterwards."""
        model = self.model
        model.train()
        user_emb, item_emb, gcnEmbedsLst, hyperEmbedsLst = model(keep_rate=1 - self.dropRate)
        # the gathers + bpr_loss of :84-88 as one op on the encoder's table (functional.
        # bpr_loss_rows; the reference's torch ops when the tables are not one device block)
        loss_rec, anchor_emb, pos_emb = bpr_loss_rows(user_emb, item_emb, user_idx, pos_idx,
                                                      neg_idx)
        loss_ssl = self.ssl_loss(anchor_emb, pos_emb, gcnEmbedsLst, hyperEmbedsLst)
        batch_loss = loss_rec + loss_ssl
        self.optimizer.zero_grad()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 4)  # before backward, as :95
        batch_loss.backward()
        return batch_loss

    def graph_step(self, user_idx, pos_idx, neg_idx) -> torch.Tensor:
        """:meth:`train_step`, replayed from a HIP graph in graph mode: the first full-size batch
        runs eagerly (a real step that also allocates the optimizer state), the second is
        recorded (recording runs nothing) and replayed, every later full-size batch replays;
        a short last batch runs eagerly (its shapes differ)."""
        if not getattr(self, "graph_mode", False):  # (subclasses with their own __init__)
            return self.train_step(user_idx, pos_idx, neg_idx)
        full = user_idx.numel() == self.batchSize
        cap = self._captured
        if cap is not None and not full:  # a short last batch runs eagerly: masks drawn inline
            self.model.edgeDropper.host_fed(False)
            out = self.train_step(user_idx, pos_idx, neg_idx).detach()
            self.model.edgeDropper.host_fed(not self.model.edgeDropper.device_rng)
            return out
        if cap is not None and full:
            return self._replay(user_idx, pos_idx, neg_idx)
        if cap is None and full and getattr(self, "_eager_steps", 0) >= 1:
            from .graphs import CapturedStep
            dropper = self.model.edgeDropper
            host_fed = not dropper.device_rng
            # the capture records the slots; refill() fills them — two slot banks and one
            # captured step per bank on the reference's stream, so the draw worker's copy of
            # the next step's masks goes straight into the bank the current replay does not read
            dropper.host_fed(host_fed, banks=2 if host_fed else 1)
            opt = self.optimizer
            if self._adam_kernel:  # the graph holds the Adam kernel; its scalars come per replay
                def body(u, i, j):
                    loss = self.forward_backward(u, i, j)
                    opt.launch()
                    return loss

                def before():
                    if host_fed:
                        dropper.refill()
                    opt.prepare()
            else:
                body = self.train_step if self._adam_in_graph else self.forward_backward
                before = dropper.refill if host_fed else None
            self._captured, self._graph_grads = [], []
            for b in range(2 if host_fed and dropper._banks else 1):
                if host_fed and dropper._banks:
                    dropper.use_bank(b)
                self._captured.append(CapturedStep(body, (user_idx, pos_idx, neg_idx),
                                                   before_replay=before))
                # the gradient buffers this graph's replays write (an eager short batch
                # rebinds .grad)
                self._graph_grads.append([p.grad for p in self.model.parameters()])
            return self._replay(user_idx, pos_idx, neg_idx)
        self._eager_steps = getattr(self, "_eager_steps", 0) + 1
        # detached: a caller holding the loss would keep the eager autograd graph — and with it
        # the parameters' AccumulateGrad nodes, bound to the eager stream — alive into the capture
        return self.train_step(user_idx, pos_idx, neg_idx).detach()

    def _replay(self, user_idx, pos_idx, neg_idx) -> torch.Tensor:
        b = self.model.edgeDropper.upcoming_bank() if len(self._captured) > 1 else 0
        out = self._captured[b](user_idx, pos_idx, neg_idx).detach().clone()
        if not self._adam_in_graph:  # the reference's Adam on the replay's gradients
            for p, g in zip(self.model.parameters(), self._graph_grads[b]):
                p.grad = g
            self.optimizer.step()
        return out

    def train(self, load_pretrained=False):  # HCCF.py:72-118
        model = self.model
        recall_list = []
        train_losses = []  # never reset: the scheduler sees the running mean, as the reference
        lst_performances = []
        for ep in range(self.maxEpoch):
            s_train = time.time()
            step_losses = []
            for n, batch in enumerate(next_batch_pairwise(self.data, self.batchSize,
                                                          device=self.device)):
                user_idx, pos_idx, neg_idx = batch
                step_losses.append(self.graph_step(user_idx, pos_idx, neg_idx).detach())
            # the batch losses (HCCF.py:91) feed only the epoch's mean (:115): read once here
            # instead of per batch, so the host prepares batch n+1 while the device runs batch n
            if step_losses:
                train_losses.extend(torch.stack(step_losses).tolist())
            # the fused BPR clamps out-of-range ids where the reference's gather raises: one
            # read of its device count per epoch
            bad = bpr_index_errors(self.device)
            if bad:
                raise IndexError(f"HCCF: {bad} batch rows held a user / item id out of range "
                                 f"(epoch {ep})")
            tr_time = time.time() - s_train
            model.eval()
            with torch.no_grad():
                self.user_emb, self.item_emb, _, _ = model(keep_rate=1)
                s_eval = time.time()
                cur_data, data_ep = self.fast_evaluation(ep, train_time=tr_time)
                lst_performances.append(data_ep)
                print(data_ep)
                recall_list.append(float(cur_data[2].split(':')[1]))
                _, should_stop = early_stopping(recall_list, self.early_stopping_steps)
                if should_stop:
                    break
            self.scheduler.step(np.mean(train_losses))
            print("Eval time: %f s" % (time.time() - s_eval))
        self.save_perfomance_training(lst_performances)
        self.user_emb, self.item_emb = self.best_user_emb, self.best_item_emb

    def save(self):
        with torch.no_grad():
            self.best_user_emb, self.best_item_emb, _, _ = self.model(keep_rate=1)
            print("Saving")
            self.save_model(self.model)

    def predict(self, u):
        user_id = self.data.get_user_id(u)
        score = torch.matmul(self.user_emb[user_id], self.item_emb.transpose(0, 1))
        return score.cpu().numpy()


class HGNNModel(nn.Module):
    """HGNN_HD4.HGNNModel (HGNN_HD4.py:253-335; HGNN_HD3.py:268-350 is the same class around
    its own LocalAwareEncoder), local encoder only."""

    def __init__(self, data, args, device, local_encoder=LocalAwareEncoder):
        super().__init__()
        self.data = data
        self.device = device
        self.sparse_norm_adj = sparse_tensor_of(data.norm_adj, device)
        self.p = args['p']
        self.drop_rate = args['drop_rate']
        self.layers = args['n_layers']
        self.emb_size = int(args['input_dim'])
        self.hyper_size = int(args['hyper_dim'])
        self.hyper_dim = int(args['hyper_dim'])
        self.batchSize = int(args['batch_size'])
        init = nn.init.xavier_uniform_
        self.embedding_dict = nn.ParameterDict({
            'user_emb': nn.Parameter(init(torch.empty(data.n_users, self.hyper_dim)).to(device)),
            'item_emb': nn.Parameter(init(torch.empty(data.n_items, self.hyper_dim)).to(device)),
        })
        self.hgnn_layer_local = local_encoder(data, self.emb_size, self.hyper_size,
                                              self.layers, self.p, self.drop_rate, device)
        self.act = nn.LeakyReLU(self.p)
        self.dropout = nn.Dropout(self.drop_rate)
        self.edgeDropper = SpAdjDropEdge()

    def forward(self, mode='local', keep_rate=1):
        if mode != 'local':
            raise NotImplementedError("HGNN_HD4: only the local (ED-HNN) encoder is built; the "
                                      "reference's group encoder is broken as shipped")
        ego = torch.cat([self.embedding_dict['user_emb'], self.embedding_dict['item_emb']], 0)
        adj = self.edgeDropper(self.sparse_norm_adj, keep_rate)
        return self.hgnn_layer_local(ego, adj)

    def calculate_cf_loss(self, anchor_emb, pos_emb, neg_emb, reg):  # :324-328
        rec_loss = bpr_loss(anchor_emb, pos_emb, neg_emb)
        reg_loss = l2_reg_loss(reg, anchor_emb, pos_emb, neg_emb) / self.batchSize
        return rec_loss + reg_loss


class HGNN_HD4(GraphRecommender):
    """model/graph/HGNN_HD4.py:32-251, ``--mode=local_only``."""

    local_encoder = LocalAwareEncoder

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        GraphRecommender.__init__(self, conf, training_set, test_set, knowledge_set, **kwargs)
        self._parse_config(kwargs)
        if self.mode != 'local_only':
            raise NotImplementedError(
                f"{type(self).__name__} --mode={self.mode}: only local_only is supported (the "
                "reference's "
                "group-aware encoder is broken as shipped, HGNN_HD4.py:320-322, :430)")
        self.set_seed()
        self.model = HGNNModel(self.data, kwargs, self.device,
                               self.local_encoder).to(self.device)
        self.model.edgeDropper.device_rng = bool(kwargs.get('hgd_device_rng', False))
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=self.lRate,
                                          weight_decay=self.weight_decay)
        self.scheduler = ReduceLROnPlateau(self.optimizer, 'min', factor=self.lr_decay,
                                           patience=10)

    def _parse_config(self, kwargs):  # :44-79
        self.dataset = kwargs['dataset']
        self.lRate = float(kwargs['lrate'])
        self.lr_decay = float(kwargs['lr_decay'])
        self.maxEpoch = int(kwargs['max_epoch'])
        self.batchSize = int(kwargs['batch_size'])
        self.reg = float(kwargs['reg'])
        self.hyper_dim = int(kwargs['hyper_dim'])
        self.p = float(kwargs['p'])
        self.drop_rate = float(kwargs['drop_rate'])
        self.layers = int(kwargs['n_layers'])
        self.cl_rate = float(kwargs['cl_rate'])
        self.temp = kwargs['temp']
        self.seed = kwargs['seed']
        self.mode = kwargs['mode']
        self.early_stopping_steps = kwargs['early_stopping_steps']
        self.weight_decay = kwargs['weight_decay']

    def set_seed(self):  # :81-92
        seed = self.seed
        np.random.seed(seed)
        random.seed(seed)
        torch.manual_seed(seed)
        torch.cuda.manual_seed(seed)
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False
        os.environ["PYTHONHASHSEED"] = str(seed)
        print(f"Random seed set as {seed}")

    def train(self, load_pretrained=False):  # :94-225 (local_only branch)
        train_model = self.model
        lst_train_losses, lst_cf_losses, lst_cl_losses = [], [], []
        lst_performances, recall_list = [], []
        for ep in range(self.maxEpoch):
            cf_losses = []
            cf_total_loss = 0
            n_cf_batch = int(self.data.n_cf_train // self.batchSize + 1)
            train_model.train()
            s_train = time.time()
            for n, batch in enumerate(next_batch_pairwise(self.data, self.batch_size,
                                                          device=self.device)):
                user_idx, pos_idx, neg_idx = batch
                user_emb_lc, item_emb_lc = train_model(mode='local', keep_rate=1 - self.drop_rate)
                cf_batch_loss = train_model.calculate_cf_loss(
                    user_emb_lc[user_idx], item_emb_lc[pos_idx], item_emb_lc[neg_idx], self.reg)
                cf_total_loss += cf_batch_loss.item()
                self.optimizer.zero_grad()
                cf_batch_loss.backward()
                self.optimizer.step()
                cf_losses.append(cf_batch_loss.item())
                if (n % 20) == 0:
                    print('CF Training: Epoch {:04d} Iter {:04d} / {:04d} | Iter Loss {:.4f} | '
                          'Iter Mean Loss {:.4f}'.format(ep, n, n_cf_batch, cf_batch_loss.item(),
                                                         cf_total_loss / (n + 1)))
                # the reference does the epoch bookkeeping inside the batch loop (:171-189):
                # scheduler step on the running mean and eval() after every batch
                cf_loss = np.mean(cf_losses)
                train_time = time.time() - s_train
                lst_cf_losses.append([ep, cf_loss])
                lst_train_losses.append([ep, cf_loss])
                lst_cl_losses.append([ep, 0])
                self.scheduler.step(cf_loss)
                train_model.eval()
            with torch.no_grad():
                self.user_emb, self.item_emb = train_model(mode='local')
                cur_data, data_ep = self.fast_evaluation(ep, train_time=train_time)
                lst_performances.append(data_ep)
                recall_list.append(float(cur_data[2].split(':')[1]))
                _, should_stop = early_stopping(recall_list, self.early_stopping_steps)
                if should_stop:
                    break
        self.save_loss(lst_train_losses, lst_cf_losses, lst_cl_losses)
        self.save_perfomance_training(lst_performances)
        self.user_emb, self.item_emb = self.best_user_emb, self.best_item_emb

    def predict(self, u):
        user_id = self.data.get_user_id(u)
        score = torch.matmul(self.user_emb[user_id], self.item_emb.transpose(0, 1))
        return score.cpu().numpy()

    def save(self):
        with torch.no_grad():
            self.best_user_emb, self.best_item_emb = self.model.forward(mode='local')
            self.save_model(self.model)


class HGNN_HD3(HGNN_HD4):
    """model/graph/HGNN_HD3.py:37-266: HGNN_HD4's plugin code line for line (plus
    ``torch.cuda.manual_seed_all`` in set_seed) around the SpMM-form local encoder."""

    local_encoder = LocalAwareEncoderHD3

    def set_seed(self):  # HGNN_HD3.py:86-98
        torch.cuda.manual_seed_all(self.seed)
        super().set_seed()


class HGCN_Encoder(nn.Module):
    """HGCN.py:104-164: per layer a TransformerEncoder over all nodes (batch 1), then HGCNConv
    on the edge-dropped norm_adj (LeakyReLU except the last layer), plus the input residual.
    As in the reference the transformer / conv layers live in plain lists (not registered)."""

    def __init__(self, data, emb_size, hyper_size, n_layers, leaky, drop_rate, device):
        super().__init__()
        self.data = data
        self.latent_size = emb_size
        self.hyper_size = hyper_size
        self.layers = n_layers
        self.norm_adj = data.norm_adj
        init = nn.init.xavier_uniform_
        self.embedding_dict = nn.ParameterDict({
            'user_emb': nn.Parameter(init(torch.empty(data.n_users, hyper_size))),
            'item_emb': nn.Parameter(init(torch.empty(data.n_items, hyper_size))),
        })
        self.sparse_norm_adj = sparse_tensor_of(self.norm_adj, device)
        self.relu = nn.ReLU()
        self.act = nn.LeakyReLU(leaky)
        self.dropout = nn.Dropout(drop_rate)
        self.edgeDropper = SpAdjDropEdge()
        self.residuals = torch.nn.ModuleList()
        self.hgnn_layers = []
        self.ugformer_layers = []
        for _ in range(self.layers):
            enc = nn.TransformerEncoderLayer(d_model=hyper_size, nhead=2, dim_feedforward=32,
                                             dropout=drop_rate)
            self.ugformer_layers.append(
                nn.TransformerEncoder(enc, 1, norm=nn.LayerNorm(hyper_size)).to(device))
            self.hgnn_layers.append(HGCNConv(leaky=leaky))

    def forward(self, keep_rate=1):
        ego = torch.cat([self.embedding_dict['user_emb'], self.embedding_dict['item_emb']], 0)
        adj = self.edgeDropper(self.sparse_norm_adj, keep_rate)
        res = ego
        all_embeddings = []
        for k in range(self.layers):
            ego = torch.squeeze(self.ugformer_layers[k](torch.unsqueeze(ego, 1)), 1)
            if k != self.layers - 1:
                ego = self.hgnn_layers[k](adj, ego)
            else:
                ego = self.hgnn_layers[k](adj, ego, act=False)
            all_embeddings += [ego]
        all_embeddings[-1] = all_embeddings[-1] + res
        nu = self.data.n_users
        return split_rows(all_embeddings[-1], nu)


class HGCN(GraphRecommender):
    """model/graph/HGCN.py:15-102."""

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        super().__init__(conf, training_set, test_set, knowledge_set, **kwargs)
        self.n_layers = int(kwargs['n_layers'])
        self.early_stopping_steps = int(kwargs['early_stopping_steps'])
        self.weight_decay = float(kwargs['weight_decay'])
        self.emb_size = int(kwargs['input_dim'])
        self.hyper_size = int(kwargs['hyper_dim'])
        self.leaky = float(kwargs['p'])
        self.drop_rate = float(kwargs['drop_rate'])
        self.reg = float(kwargs['reg'])
        self.model = HGCN_Encoder(self.data, self.emb_size, self.hyper_size, self.n_layers,
                                  self.leaky, self.drop_rate, self.device)
        self.model.edgeDropper.device_rng = bool(kwargs.get('hgd_device_rng', False))

    def train(self, load_pretrained=False):
        model = self.model.to(self.device)
        optimizer = torch.optim.Adam(model.parameters(), lr=self.lRate,
                                     weight_decay=self.weight_decay)
        scheduler = ReduceLROnPlateau(optimizer, 'min', factor=self.lr_decay, patience=10)
        recall_list = []
        lst_train_losses, lst_rec_losses, lst_reg_losses, lst_performances = [], [], [], []
        for epoch in range(self.maxEpoch):
            train_losses, rec_losses, reg_losses = [], [], []
            for n, batch in enumerate(next_batch_pairwise(self.data, self.batch_size,
                                                          device=self.device)):
                user_idx, pos_idx, neg_idx = batch
                rec_user_emb, rec_item_emb = model(keep_rate=1 - self.drop_rate)
                user_emb = rec_user_emb[user_idx]
                pos_item_emb, neg_item_emb = rec_item_emb[pos_idx], rec_item_emb[neg_idx]
                rec_loss = bpr_loss(user_emb, pos_item_emb, neg_item_emb)
                reg_loss = l2_reg_loss(self.reg, user_emb, pos_item_emb,
                                       neg_item_emb) / self.batch_size
                batch_loss = rec_loss + reg_loss
                train_losses.append(batch_loss.item())
                rec_losses.append(rec_loss.item())
                reg_losses.append(reg_loss.item())
                optimizer.zero_grad()
                batch_loss.backward()
                optimizer.step()
                if n % 100 == 0 and n > 0:
                    print('training:', epoch + 1, 'batch', n, 'batch_loss:', batch_loss.item())
            train_loss = np.mean(train_losses)
            scheduler.step(train_loss)
            lst_train_losses.append([epoch, train_loss])
            lst_rec_losses.append([epoch, np.mean(rec_losses)])
            lst_reg_losses.append([epoch, np.mean(reg_losses)])
            with torch.no_grad():
                self.user_emb, self.item_emb = model()
            measure, data_ep = self.fast_evaluation(epoch)
            lst_performances.append(data_ep)
            recall_list.append(float(measure[2].split(':')[1]))
            _, should_stop = early_stopping(recall_list, self.early_stopping_steps)
            if should_stop:
                break
        self.save_loss(lst_train_losses, lst_rec_losses, lst_reg_losses)
        self.save_perfomance_training(lst_performances)
        self.user_emb, self.item_emb = self.best_user_emb, self.best_item_emb

    def save(self):
        with torch.no_grad():
            self.best_user_emb, self.best_item_emb = self.model.forward()
            self.save_model(self.model)

    def predict(self, u):
        u = self.data.get_user_id(u)
        score = torch.matmul(self.user_emb[u], self.item_emb.transpose(0, 1))
        return score.cpu().numpy()


class _ShardedPlugin:
    """What the sharded plugins share: the rank's user range, global-id row assembly by
    differentiable all-reduce, the full user table for evaluation, rank-0 file output."""

    def _init_dist(self):
        import torch.distributed as dist
        from .sharded import all_reduce_sum
        from .sharded_encoders import shard_bounds
        if not dist.is_initialized():
            raise RuntimeError(f"{type(self).__name__}: torch.distributed is not initialised")
        self._dist, self._all_reduce_sum = dist, all_reduce_sum
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.is_main = self.rank == 0
        # degree-balanced contiguous user ranges (every rank derives the same cuts from the data)
        deg = np.diff(self.data.interaction_mat.tocsr().indptr)
        self.u0, self.u1 = shard_bounds(self.data.n_users, self.world, self.rank, deg)
        self._sync_host_rng()

    def _sync_host_rng(self):
        """Every rank must draw the same global batch (the sampler shuffles and samples with
        Python's ``random``) and the same CPU drop-edge mask (torch's CPU generator): rank 0's
        Python, numpy and torch-CPU generator states are broadcast to all ranks. The per-rank
        CUDA generators are left alone (per-rank dropout masks, sharded_encoders)."""
        import random
        dist = self._dist
        box = [(random.getstate(), np.random.get_state(), torch.get_rng_state())]
        dist.broadcast_object_list(box, src=0)
        py, npy, th = box[0]
        random.setstate(py)
        np.random.set_state(npy)
        torch.set_rng_state(th)

    def _check_batch(self, *idx: torch.Tensor) -> None:
        """Raises if the ranks do not hold the same global batch: one all-reduce of a position-
        weighted checksum of the index tensors (MAX of (c, -c) equal to (c, -c) on every rank)."""
        c = sum(int(k + 1) * (t.to(torch.int64) * torch.arange(
            1, t.numel() + 1, device=t.device)).sum() for k, t in enumerate(idx))
        v = torch.stack([c, -c]).to(torch.int64)
        m = v.clone()
        from .sharded import ordered_all_reduce
        ordered_all_reduce(m, op=self._dist.ReduceOp.MAX)
        if not torch.equal(m, v):
            raise RuntimeError(f"{type(self).__name__}: ranks drew different batches (the "
                               "Python random state diverged); the sharded loss would be wrong")

    def _rows(self, table_local: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
        """table[ids] for GLOBAL user ids (negative ids wrap, as torch indexing) of a user table
        sharded by rows: each owner contributes its rows, the rest zeros, summed over ranks."""
        return self._rows_multi([table_local], ids)[0]

    def _rows_multi(self, tables_local, ids: torch.Tensor):
        """``[t[ids] for t in tables_local]`` for several user tables sharded alike, with ONE
        (differentiable) all-reduce of the stacked owner parts instead of one per table."""
        n = self.data.n_users
        d = tables_local[0].shape[1]
        if self.u1 == self.u0:  # a rank without users contributes nothing
            part = torch.zeros(len(tables_local) * ids.numel(), d, device=ids.device)
        else:
            g = torch.where(ids < 0, ids + n, ids)
            own = (g >= self.u0) & (g < self.u1)
            loc = (g - self.u0).clamp(0, max(self.u1 - self.u0 - 1, 0))
            zero = torch.zeros((), device=ids.device)
            part = torch.cat([torch.where(own[:, None], t[loc], zero) for t in tables_local], 0)
        return list(self._all_reduce_sum(part).split(ids.numel(), 0))

    def _full_user_table(self, user_local: torch.Tensor) -> torch.Tensor:
        full = torch.zeros(self.data.n_users, user_local.shape[1], device=user_local.device)
        full[self.u0:self.u1] = user_local
        from .sharded import ordered_all_reduce
        ordered_all_reduce(full)
        return full


    def _backward_step(self, loss: torch.Tensor, replicated) -> None:
        """Every rank holds the same full loss: backward of loss/world, then the replicated
        parameters' partial gradients summed over ranks, then the optimizer step."""
        from .sharded import allreduce_replicated_grads
        (loss / self.world).backward()
        allreduce_replicated_grads(replicated)
        self.optimizer.step()

    def save_model(self, model):
        if self.is_main:  # every rank holds its own user rows: rank 0 saves its shard's state
            super().save_model(model)

    def save_perfomance_training(self, log_train):
        if self.is_main:
            super().save_perfomance_training(log_train)

    def save_loss(self, *a, **k):
        if self.is_main:
            super().save_loss(*a, **k)

    def evaluate(self, rec_list):
        if self.is_main:
            return super().evaluate(rec_list)
        # the other ranks hold the same measures, without writing the files
        from .evaluation import ranking_evaluation
        _, ids, _ = self._device_eval()
        self.result = ranking_evaluation(self._tests, ids, self.topN)


class HCCF_sharded(_ShardedPlugin, HCCF):
    """HCCF's training loop (HCCF.py:72-118) on user-row shards, one process per GPU under
    ``torch.distributed`` (backend "nccl" = RCCL over xGMI). Not a reference model
    name: the reference has no distributed code; this is the north_star's user-row partition
    carried up to the plugin.

    Every rank builds the data, runs the same sampler (same Python random state, so the same
    global batch) and holds ``sharded_encoders.ShardedHCCFEncoder`` (its users' rows; items and
    W replicated, broadcast from rank 0 at start). A step computes the reference's loss exactly:
    the batch's anchor rows and the user rows the InfoNCE node list picks are assembled on every
    rank by a differentiable all-reduce of each owner's rows, so every rank evaluates the same
    full loss; its backward is scaled by 1/world, which makes the per-rank gradients of the
    replicated parameters the partials that ``allreduce_replicated_grads`` sums (and the
    all-reduce's backward gives each owner its rows' full gradient). Evaluation all-reduces the
    user table once per epoch and runs the single-GPU device evaluation; rank 0 writes the
    result files. With ``drop_rate`` 0 and the reference's CPU drop-edge stream it takes the
    same steps as :class:`HCCF` on one GPU (``tests/test_gpu_plugins.py``)."""

    _graph_default = False  # its steps all-reduce: no graph replay

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        from .sharded_encoders import ShardedHCCFEncoder
        GraphRecommender.__init__(self, conf, training_set, test_set, knowledge_set, **kwargs)
        self._init_dist()
        dist = self._dist
        self._parse_config(self.config, kwargs)
        self.model = ShardedHCCFEncoder(kwargs, self.data, self.u0, self.u1, device=self.device,
                                        device_rng=bool(kwargs.get('hgd_device_rng', False)),
                                        seed=self.seed)
        from .sharded import ordered_broadcast
        with torch.no_grad():  # replicated parameters start equal on every rank
            for p in self.model.replicated_parameters():
                ordered_broadcast(p.data, 0)
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=self.lRate)
        self.scheduler = ReduceLROnPlateau(self.optimizer, 'min', factor=self.lr_decay,
                                           patience=5)

    def train_step(self, user_idx, pos_idx, neg_idx) -> torch.Tensor:
        model = self.model
        model.train()
        self._check_batch(user_idx, pos_idx, neg_idx)
        nl = self.u1 - self.u0
        user_emb, item_emb, gcnEmbedsLst, hyperEmbedsLst = model(keep_rate=1 - self.dropRate)
        anchor_emb = self._rows(user_emb, user_idx)
        pos_emb = item_emb[pos_idx]
        neg_emb = item_emb[neg_idx]
        bprLoss = bpr_loss(anchor_emb, pos_emb, neg_emb)
        u_nodes, p_nodes = unique_long(anchor_emb), unique_long(pos_emb)
        k = torch.arange(u_nodes.numel(), device=u_nodes.device)
        # the InfoNCE user rows of every layer (both tables) in ONE all-reduce: 2 exchanges per
        # step (the anchor rows, then these) instead of 1 + 2L. Not one: the node list is
        # torch.unique(anchor_emb.long()) (HCCF.py:65), which needs the gathered anchor rows
        e1s = [gcnEmbedsLst[i].detach() for i in range(self.nLayers)]
        e2s = list(hyperEmbedsLst[:self.nLayers])
        rows = self._rows_multi([e[:nl] for e in e1s] + [e[:nl] for e in e2s], u_nodes)
        L = self.nLayers
        sslLoss = 0
        for i in range(L):
            e1, e2 = e1s[i], e2s[i]
            sslLoss += contrast_loss(rows[i], rows[L + i], k, self.temp) \
                + contrast_loss(e1[nl:], e2[nl:], p_nodes, self.temp)
        batch_loss = bprLoss + sslLoss * self.ss_rate
        self.optimizer.zero_grad()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 4)  # before backward, as HCCF.py:95
        self._backward_step(batch_loss, model.replicated_parameters())
        return batch_loss

    def train(self, load_pretrained=False):
        model = self.model
        recall_list, train_losses, lst_performances = [], [], []
        for ep in range(self.maxEpoch):
            s_train = time.time()
            for batch in next_batch_pairwise(self.data, self.batchSize, device=self.device):
                train_losses.append(self.train_step(*batch).item())
            tr_time = time.time() - s_train
            model.eval()
            with torch.no_grad():
                ue, self.item_emb, _, _ = model(keep_rate=1)
                self.user_emb = self._full_user_table(ue)
                cur_data, data_ep = self.fast_evaluation(ep, train_time=tr_time)
                lst_performances.append(data_ep)
                recall_list.append(float(cur_data[2].split(':')[1]))
                _, should_stop = early_stopping(recall_list, self.early_stopping_steps)
                if should_stop:
                    break
            self.scheduler.step(np.mean(train_losses))
        self.save_perfomance_training(lst_performances)
        self.user_emb, self.item_emb = self.best_user_emb, self.best_item_emb

    def save(self):
        with torch.no_grad():
            ue, self.best_item_emb, _, _ = self.model(keep_rate=1)
            self.best_user_emb = self._full_user_table(ue)
            self.save_model(self.model)


class ShardedHGNNModel(nn.Module):
    """HGNNModel (HGNN_HD4.py:253-335, local encoder) on user-row shards: ``user_emb`` holds this
    rank's rows, ``item_emb`` and every encoder weight are replicated."""

    def __init__(self, data, args, device, u0, u1, device_rng=False, local_encoder=None):
        super().__init__()
        from .sharded_encoders import ShardedLocalAwareEncoder
        local_encoder = local_encoder or ShardedLocalAwareEncoder
        self.data = data
        self.p = args['p']
        self.drop_rate = args['drop_rate']
        self.layers = args['n_layers']
        self.emb_size = int(args['input_dim'])
        self.hyper_size = int(args['hyper_dim'])
        self.hyper_dim = int(args['hyper_dim'])
        self.batchSize = int(args['batch_size'])
        self.device_rng = device_rng
        U, d = data.n_users, self.hyper_dim
        bu = (6.0 / (U + d)) ** 0.5  # xavier_uniform_ bound of the GLOBAL [U, d] table
        self.embedding_dict = nn.ParameterDict({
            'user_emb': nn.Parameter(torch.empty(u1 - u0, d, device=device).uniform_(-bu, bu)),
            'item_emb': nn.Parameter(nn.init.xavier_uniform_(
                torch.empty(data.n_items, d)).to(device)),
        })
        self.hgnn_layer_local = local_encoder(
            data, self.emb_size, self.hyper_size, self.layers, self.p, self.drop_rate, u0, u1,
            device=device)

    def replicated_parameters(self):
        return [self.embedding_dict['item_emb']] + list(self.hgnn_layer_local.parameters())

    def forward(self, mode='local', keep_rate=1):
        if mode != 'local':
            raise NotImplementedError("only the local (ED-HNN) encoder is built")
        ego = torch.cat([self.embedding_dict['user_emb'], self.embedding_dict['item_emb']], 0)
        enc = self.hgnn_layer_local
        return enc(ego, enc.dropped(keep_rate, self.device_rng))


class HGNN_HD4_sharded(_ShardedPlugin, HGNN_HD4):
    """HGNN_HD4 ``local_only`` (the ED-HNN "hypergraph diffusion" model; BASELINE configs[3]:
    Amazon-Book, user-row sharded on the GPUs of one node) on user-row shards under
    torch.distributed, with :class:`HCCF_sharded`'s scheme: same global batch on every rank,
    anchor rows assembled by a differentiable all-reduce, the full BPR + L2 loss on every rank,
    backward scaled by 1/world, replicated gradients (item table and every encoder weight)
    summed. The loop keeps HGNN_HD4's quirks (scheduler step and ``eval()`` inside the batch
    loop)."""

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        GraphRecommender.__init__(self, conf, training_set, test_set, knowledge_set, **kwargs)
        self._parse_config(kwargs)
        if self.mode != 'local_only':
            raise NotImplementedError(f"{type(self).__name__} --mode={self.mode}: only "
                                      "local_only is supported")
        self._init_dist()
        self.set_seed()
        self.model = ShardedHGNNModel(self.data, kwargs, self.device, self.u0, self.u1,
                                      bool(kwargs.get('hgd_device_rng', False)),
                                      self.sharded_encoder())
        from .sharded import ordered_broadcast
        with torch.no_grad():
            for p in self.model.replicated_parameters():
                ordered_broadcast(p.data, 0)
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=self.lRate,
                                          weight_decay=self.weight_decay)
        self.scheduler = ReduceLROnPlateau(self.optimizer, 'min', factor=self.lr_decay,
                                           patience=10)

    @staticmethod
    def sharded_encoder():
        from .sharded_encoders import ShardedLocalAwareEncoder
        return ShardedLocalAwareEncoder

    def cf_loss(self, anchor_emb, pos_emb, neg_emb):  # HGNNModel.calculate_cf_loss (:324-328)
        rec_loss = bpr_loss(anchor_emb, pos_emb, neg_emb)
        reg_loss = l2_reg_loss(self.reg, anchor_emb, pos_emb, neg_emb) / self.model.batchSize
        return rec_loss + reg_loss

    def train_step(self, user_idx, pos_idx, neg_idx) -> torch.Tensor:
        """One batch of HGNN_HD4.py:118-160 (local_only): BPR + L2 over the global batch."""
        self._check_batch(user_idx, pos_idx, neg_idx)
        user_emb_lc, item_emb_lc = self.model(mode='local', keep_rate=1 - self.drop_rate)
        anchor = self._rows(user_emb_lc, user_idx)
        loss = self.cf_loss(anchor, item_emb_lc[pos_idx], item_emb_lc[neg_idx])
        self.optimizer.zero_grad()
        self._backward_step(loss, self.model.replicated_parameters())
        return loss

    def train(self, load_pretrained=False):  # HGNN_HD4.py:94-225, local_only
        train_model = self.model
        lst_train_losses, lst_cf_losses, lst_cl_losses = [], [], []
        lst_performances, recall_list = [], []
        for ep in range(self.maxEpoch):
            cf_losses = []
            train_model.train()
            s_train = time.time()
            for batch in next_batch_pairwise(self.data, self.batch_size, device=self.device):
                cf_losses.append(self.train_step(*batch).item())
                cf_loss = np.mean(cf_losses)
                train_time = time.time() - s_train
                lst_cf_losses.append([ep, cf_loss])
                lst_train_losses.append([ep, cf_loss])
                lst_cl_losses.append([ep, 0])
                self.scheduler.step(cf_loss)
                train_model.eval()
            with torch.no_grad():
                ue, self.item_emb = train_model(mode='local')
                self.user_emb = self._full_user_table(ue)
                cur_data, data_ep = self.fast_evaluation(ep, train_time=train_time)
                lst_performances.append(data_ep)
                recall_list.append(float(cur_data[2].split(':')[1]))
                _, should_stop = early_stopping(recall_list, self.early_stopping_steps)
                if should_stop:
                    break
        self.save_loss(lst_train_losses, lst_cf_losses, lst_cl_losses)
        self.save_perfomance_training(lst_performances)
        self.user_emb, self.item_emb = self.best_user_emb, self.best_item_emb

    def save(self):
        with torch.no_grad():
            ue, self.best_item_emb = self.model.forward(mode='local')
            self.best_user_emb = self._full_user_table(ue)
            self.save_model(self.model)


class HGNN_HD3_sharded(HGNN_HD4_sharded):
    """HGNN_HD3 ``local_only`` (HGNN_HD3.py:37-266: HGNN_HD4's loop around the SpMM-form ED-HNN
    encoder) on user-row shards, with :class:`HGNN_HD4_sharded`'s scheme;
    ``sharded_encoders.ShardedLocalAwareEncoderHD3`` runs its blocks' HGCNConv two-hops on the
    edge-dropped ``norm_adj`` shard."""

    @staticmethod
    def sharded_encoder():
        from .sharded_encoders import ShardedLocalAwareEncoderHD3
        return ShardedLocalAwareEncoderHD3

    def set_seed(self):  # HGNN_HD3.py:86-98
        torch.cuda.manual_seed_all(self.seed)
        super().set_seed()


class HCCF_diffusion(HCCF):
    """model/graph/HCCF_diffusion.py:22-129: HCCF's constructor, losses and loop verbatim, with
    the encoder whose hypergraph hop is the ED-HNN block on the learned hypergraph."""

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        GraphRecommender.__init__(self, conf, training_set, test_set, knowledge_set, **kwargs)
        self.model = HCCFDiffusionEncoder(kwargs, self.data, self.device)
        _device_drop_edge(self.model.edgeDropper, kwargs)
        self._parse_config(self.config, kwargs)
        self.model.to(self.device)
        self._init_optimizer(kwargs)  # hgd_graph as HCCF's (the ED-HNN block is capture-safe)


class DHCF_Encoder(nn.Module):
    """DHCF.py:146-185. The reference densifies ``interaction_mat`` [U, I] and runs
    HGCNConv (``leaky(A·(Aᵀ·E_u))`` for users, ``leaky(Aᵀ·(A·E_i))`` for items) on it with
    torch.sparse.mm; here the same operator runs on the sparse matrix (values = interaction
    counts, as the dense copy holds them). Every layer applies the conv to the layer-0
    embeddings (the reference passes ``uEmbed`` / ``iEmbed`` each time), so all layers are the
    same tensor: it is computed once and concatenated L times — identical values, and autograd
    sums the L copies' gradients exactly as it sums the reference's L identical branches.
    ``fc_u`` / ``fc_i`` exist (and are optimised) but are unused, as in the reference."""

    def __init__(self, config, data, args, device):
        super().__init__()
        self.data = data
        self.input_dim = args['input_dim']
        self.hyper_dim = args['hyper_dim']
        self.p = args['p']
        self.drop_rate = args['drop_rate']
        self.layers = args['n_layers']
        self.adj = sparse_tensor_of(data.interaction_mat, device)        # [U, I]
        self.adj_t = sparse_tensor_of(data.interaction_mat.T.tocsr(), device)  # [I, U]
        init = nn.init.xavier_uniform_
        self.embedding_dict = nn.ParameterDict({
            'user_emb': nn.Parameter(init(torch.empty(data.n_users, self.hyper_dim)).to(device)),
            'item_emb': nn.Parameter(init(torch.empty(data.n_items, self.hyper_dim)).to(device)),
        })
        self.fc_u = nn.Linear(self.hyper_dim, self.hyper_dim)
        self.fc_i = nn.Linear(self.hyper_dim, self.hyper_dim)
        self.hgnn_u = HGCNConv(leaky=self.p)
        self.hgnn_i = HGCNConv(leaky=self.p)
        self.non_linear = nn.ReLU()
        self.dropout = nn.Dropout(self.drop_rate)

    def forward(self):
        uEmbed = self.embedding_dict['user_emb']
        iEmbed = self.embedding_dict['item_emb']
        hu = self.hgnn_u(self.adj, uEmbed)
        hi = self.hgnn_i(self.adj_t, iEmbed)
        return (torch.cat([uEmbed] + [hu] * self.layers, dim=1),
                torch.cat([iEmbed] + [hi] * self.layers, dim=1))


class DHCF(GraphRecommender):
    """model/graph/DHCF.py:19-130."""

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        super().__init__(conf, training_set, test_set, knowledge_set, **kwargs)
        self.kwargs = kwargs
        self.model = DHCF_Encoder(self.config, self.data, kwargs, self.device)
        self.lRate = float(kwargs['lrate'])
        self.lr_decay = float(kwargs['lr_decay'])
        self.maxEpoch = int(kwargs['max_epoch'])
        self.batchSize = int(kwargs['batch_size'])
        self.reg = float(kwargs['reg'])
        self.weight_decay = float(kwargs['weight_decay'])
        self.early_stopping_steps = int(kwargs['early_stopping_steps'])

    def train(self, load_pretrained=False):
        model = self.model.to(self.device)
        optimizer = torch.optim.Adam(model.parameters(), lr=self.lRate,
                                     weight_decay=self.weight_decay)
        scheduler = ReduceLROnPlateau(optimizer, 'min', factor=self.lr_decay, patience=5)
        lst_train_losses, lst_rec_losses, lst_reg_losses = [], [], []
        lst_performances, recall_list = [], []
        for epoch in range(self.maxEpoch):
            train_losses, rec_losses, reg_losses = [], [], []
            s_train = time.time()
            for n, batch in enumerate(next_batch_pairwise(self.data, self.batch_size,
                                                          device=self.device)):
                user_idx, pos_idx, neg_idx = batch
                rec_user_emb, rec_item_emb = model()
                user_emb = rec_user_emb[user_idx]
                pos_item_emb, neg_item_emb = rec_item_emb[pos_idx], rec_item_emb[neg_idx]
                rec_loss = bpr_loss(user_emb, pos_item_emb, neg_item_emb)
                reg_loss = l2_reg_loss(self.reg, user_emb, pos_item_emb,
                                       neg_item_emb) / self.batch_size
                batch_loss = rec_loss + reg_loss
                train_losses.append(batch_loss.item())
                rec_losses.append(rec_loss.item())
                reg_losses.append(reg_loss.item())
                optimizer.zero_grad()
                torch.nn.utils.clip_grad_norm_(model.parameters(), 4)
                batch_loss.backward()
                optimizer.step()
                if n % 100 == 0 and n > 0:
                    print('training:', epoch + 1, 'batch', n, 'batch_loss:', batch_loss.item())
            tr_time = time.time() - s_train
            train_loss = np.mean(train_losses)
            lst_train_losses.append([epoch, train_loss])
            lst_rec_losses.append([epoch, np.mean(rec_losses)])
            lst_reg_losses.append([epoch, np.mean(reg_losses)])
            scheduler.step(train_loss)
            with torch.no_grad():
                self.user_emb, self.item_emb = model()
                cur_data, data_ep = self.fast_evaluation(epoch, train_time=tr_time)
                lst_performances.append(data_ep)
                recall_list.append(float(cur_data[2].split(':')[1]))
                _, should_stop = early_stopping(recall_list, self.early_stopping_steps)
                if should_stop:
                    break
        self.save_loss(lst_train_losses, lst_rec_losses, lst_reg_losses)
        self.save_perfomance_training(lst_performances)
        self.user_emb, self.item_emb = self.best_user_emb, self.best_item_emb

    def save(self):
        with torch.no_grad():
            self.best_user_emb, self.best_item_emb = self.model.forward()
            self.save_model(self.model)

    def predict(self, u):
        u = self.data.get_user_id(u)
        score = torch.matmul(self.user_emb[u], self.item_emb.transpose(0, 1))
        return score.cpu().numpy()


PLUGINS = {"HCCF": HCCF, "HCCF_sharded": HCCF_sharded, "HGNN_HD4_sharded": HGNN_HD4_sharded,
           "HGNN_HD3_sharded": HGNN_HD3_sharded, "HGNN_HD4": HGNN_HD4, "HGNN_HD3": HGNN_HD3,
           "HGCN": HGCN, "HCCF_diffusion": HCCF_diffusion, "DHCF": DHCF}
