"""torch-CPU restatement of the hybrid CTC/attention training math (oracle; test infra only).

Pure functions over a parameter dict keyed by the REFERENCE's state_dict names,
so fixtures recorded from the reference load directly.  Gradients come from
torch autograd on CPU.  Every function cites the reference lines it restates.
Nothing here is imported by the product package.
"""
import numpy as np
import torch

from . import ctc_ref


# ---------------------------------------------------------------------------
# LSTM direction with packed-sequence semantics (rnn.py:166-172, 218-224, 343-390)
# ---------------------------------------------------------------------------
def lstm_direction(x, lens, w_ih, w_hh, b_ih, b_hh, reverse):
    """x: [B, T, Din] (sorted desc by lens).  Gate order i, f, g, o; h0 = c0 = 0
    (rnn.py:499-536).  The reverse direction starts at each utterance's own last
    frame; outputs beyond the length are zero (pack/pad_packed semantics)."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    gx = torch.matmul(x, w_ih.t()) + b_ih + b_hh            # [B, T, 4H]
    h = x.new_zeros(B, H)
    c = x.new_zeros(B, H)
    outs = [None] * T
    lens_t = torch.as_tensor(np.asarray(lens), dtype=torch.long)
    order = range(T - 1, -1, -1) if reverse else range(T)
    for t in order:
        g = gx[:, t] + h @ w_hh.t()
        i, f, gg, o = g.split(H, dim=1)
        c_new = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h_new = torch.sigmoid(o) * torch.tanh(c_new)
        act = (lens_t > t).to(x.dtype).unsqueeze(1)
        h = h_new * act
        c = c_new * act
        outs[t] = h
    return torch.stack(outs, dim=1)


def gru_direction(x, lens, w_ih, w_hh, b_ih, b_hh, reverse):
    """nn.GRU direction (rnn.py:173-191, 226-233; torch's GRU equations), gate
    order r, z, n: r = sig(W_ir x + b_ir + W_hr h + b_hr), z likewise,
    n = tanh(W_in x + b_in + r * (W_hn h + b_hn)), h' = (1 - z) n + z h; h0 = 0
    and the same packed-sequence semantics as lstm_direction."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    gx = torch.matmul(x, w_ih.t()) + b_ih                    # [B, T, 3H]
    h = x.new_zeros(B, H)
    outs = [None] * T
    lens_t = torch.as_tensor(np.asarray(lens), dtype=torch.long)
    order = range(T - 1, -1, -1) if reverse else range(T)
    for t in order:
        gh = h @ w_hh.t() + b_hh
        xr, xz, xn = gx[:, t].split(H, dim=1)
        hr, hz, hn = gh.split(H, dim=1)
        r = torch.sigmoid(xr + hr)
        z = torch.sigmoid(xz + hz)
        n = torch.tanh(xn + r * hn)
        h_new = (1 - z) * n + z * h
        h = h_new * (lens_t > t).to(x.dtype).unsqueeze(1)
        outs[t] = h
    return torch.stack(outs, dim=1)


@torch.no_grad()
def lstm_direction_bptt(x, lens, w_ih, w_hh, b_ih, b_hh, reverse, dy):
    """lstm_direction's forward plus an explicit O(T) backward (BPTT) for the
    cotangent dy [B, T, H] -- the same math as autograd through
    lstm_direction (checked in tests/test_recurrence_full.py) without
    autograd's O(T^2) slice-gradient cost, so the oracle runs at the bench
    shape (B = 32, T = 1000, H = 512) in seconds.  Computes in x's dtype.
    Returns (y [B, T, H], dx [B, T, Din], dW_ih, dW_hh, db) where db is the
    gradient of b_ih (equal to that of b_hh)."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    gx = torch.matmul(x, w_ih.t()) + b_ih + b_hh
    lens_t = torch.as_tensor(np.asarray(lens), dtype=torch.long)
    order = list(range(T - 1, -1, -1)) if reverse else list(range(T))
    h = x.new_zeros(B, H)
    c = x.new_zeros(B, H)
    y = x.new_zeros(B, T, H)
    saved = [None] * T
    for t in order:
        g = gx[:, t] + h @ w_hh.t()
        i, f, gg, o = torch.sigmoid(g[:, :H]), torch.sigmoid(g[:, H:2 * H]), \
            torch.tanh(g[:, 2 * H:3 * H]), torch.sigmoid(g[:, 3 * H:])
        c_new = f * c + i * gg
        tc = torch.tanh(c_new)
        act = (lens_t > t).to(x.dtype).unsqueeze(1)
        saved[t] = (h, c, i, f, gg, o, tc, act)
        h = o * tc * act
        c = c_new * act
        y[:, t] = h
    dgx = torch.zeros_like(gx)
    dw_hh = torch.zeros_like(w_hh)
    dh = x.new_zeros(B, H)
    dc = x.new_zeros(B, H)
    for t in reversed(order):
        h_prev, c_prev, i, f, gg, o, tc, act = saved[t]
        dh_t = (dy[:, t] + dh) * act
        dc_t = dc * act + dh_t * o * (1 - tc * tc)
        d_o = dh_t * tc * o * (1 - o)
        d_i = dc_t * gg * i * (1 - i)
        d_g = dc_t * i * (1 - gg * gg)
        d_f = dc_t * c_prev * f * (1 - f)
        dg = torch.cat([d_i, d_f, d_g, d_o], dim=1)
        dgx[:, t] = dg
        dw_hh += dg.t() @ h_prev
        dh = dg @ w_hh
        dc = dc_t * f
    dx = torch.matmul(dgx, w_ih)
    dw_ih = torch.einsum('btg,btd->gd', dgx, x)
    db = dgx.sum(dim=(0, 1))
    return y, dx, dw_ih, dw_hh, db


def vgg_front(p, prefix, cfg, xs, x_lens, masks=None, training=True, decisions=None):
    """CNNEncoder.forward (encoders/cnn.py:124-165) with relu, 3x3 / stride 1 /
    padding 1 convs, max-pool (first floor mode, later ceil mode), BatchNorm2d
    in training mode (batch statistics; running stats returned, not written)
    and optional replayed dropout masks (masks[l]: [B, T', F', C] scales).
    decisions (test infrastructure: the bf16 pins): per layer (relu_mask
    [B, C, F, T] bool, pool_index [B, C, F', T'] int64 flat index f * T + t of
    each window's maximum, or None) -- the ReLU and max-pool choices of another
    evaluation (the GPU's) replayed, so rounding-level differences of the
    activations cannot move a max-pool argmax or a ReLU sign and route the
    gradient to another pixel.
    Returns (out [B, T', F'*C], lens np.int64 via ConvOutSize's floor rule
    (cnn_utils.py:25-37), running-stat updates {name: tensor})."""
    Fn = torch.nn.functional
    x = xs.transpose(1, 2).unsqueeze(1)                       # [B, 1, F, T] (cnn.py:143-149)
    lens = np.asarray(x_lens).astype(np.int64)
    idx, first_pool, stats = 0, True, {}
    for l, C in enumerate(cfg['conv_channels']):
        conv = '%sconv.layers.%d.' % (prefix, idx)
        x = Fn.conv2d(x, p[conv + 'weight'], p.get(conv + 'bias'), stride=1, padding=1)
        idx += 2                                              # conv, relu
        x = torch.relu(x) if decisions is None else x * decisions[l][0].to(x.dtype)
        pl = cfg['poolings'][l]
        if len(pl):
            if decisions is None:
                x = Fn.max_pool2d(x, kernel_size=tuple(pl), stride=tuple(pl),
                                  ceil_mode=not first_pool)
            else:
                ind = decisions[l][1]
                x = x.flatten(2).gather(2, ind.flatten(2)).view(ind.shape)
            lens = np.floor((lens - pl[1]) / pl[1] + 1).astype(np.int64)
            first_pool = False
            idx += 1
        if cfg.get('batch_norm'):
            bn = '%sconv.layers.%d.' % (prefix, idx)
            rm = p[bn + 'running_mean'].clone()
            rv = p[bn + 'running_var'].clone()
            x = Fn.batch_norm(x, rm, rv, p[bn + 'weight'], p[bn + 'bias'], training=training,
                              momentum=0.1, eps=1e-5)
            stats[bn + 'running_mean'], stats[bn + 'running_var'] = rm, rv
            idx += 1
        if masks is not None:
            x = x * torch.from_numpy(masks[l]).permute(0, 3, 2, 1)   # [B,T',F',C] -> NCHW
        idx += 1                                              # dropout
    B, C, Fo, To = x.shape
    return x.transpose(1, 3).reshape(B, To, Fo * C), lens, stats


def vgg_decisions(p, prefix, cfg, xs, training=True):
    """The ReLU masks and max-pool argmax indices vgg_front's forward takes
    (its `decisions` format; replaying them reproduces it exactly)."""
    Fn = torch.nn.functional
    x = xs.transpose(1, 2).unsqueeze(1)
    idx, first_pool, out = 0, True, []
    for l, C in enumerate(cfg['conv_channels']):
        conv = '%sconv.layers.%d.' % (prefix, idx)
        z = Fn.conv2d(x, p[conv + 'weight'], p.get(conv + 'bias'), stride=1, padding=1)
        idx += 2
        mask = z > 0
        x = torch.relu(z)
        pl = cfg['poolings'][l]
        ind = None
        if len(pl):
            x, ind = Fn.max_pool2d(x, kernel_size=tuple(pl), stride=tuple(pl),
                                   ceil_mode=not first_pool, return_indices=True)
            first_pool = False
            idx += 1
        if cfg.get('batch_norm'):
            bn = '%sconv.layers.%d.' % (prefix, idx)
            x = Fn.batch_norm(x, p[bn + 'running_mean'].clone(), p[bn + 'running_var'].clone(),
                              p[bn + 'weight'], p[bn + 'bias'], training=training,
                              momentum=0.1, eps=1e-5)
            idx += 1
        idx += 1
        out.append((mask, ind))
    return out


def blstm_encoder(p, prefix, cfg, xs, x_lens, capture_layer=0):
    """RNNEncoder.forward (rnn.py:284-487) for rnn_type 'lstm' or 'gru'
    (cfg['rnn_type']), bidirectional,
    dropout = 0, optional VGG front-end (cfg['conv_channels'], rnn.py:314-316),
    and the inter-layer ops of rnn.py:409-465 on every layer but the last:
    projection tanh(proj_l(x)) (cfg['num_proj']), subsampling 'drop'
    x[:, 1::2] or 'concat' [x_{2t}; x_{2t+1}] (cfg['subsample_type']), residual
    / dense residual sums from layer residual_start_layer - 1 on (rnn.py:126-133).

    Returns (out [B, T', 2H], out_lens np.int32 [B], perm np.int64 [B]); with
    capture_layer = k >= 1 also (out_k, lens_k) of layer k-1 after its dropout,
    before projection / subsampling (rnn.py:400-407)."""
    x_lens = np.asarray(x_lens)
    if cfg.get('conv_channels'):
        xs, x_lens, _ = vgg_front(p, prefix, cfg, xs, x_lens,
                                  training=cfg.get('bn_training', True),
                                  decisions=cfg.get('vgg_decisions'))
    perm = np.argsort(-x_lens, kind='stable')                 # rnn.py:319-326
    xs = xs[torch.as_tensor(perm)]
    lens = x_lens[perm].astype(np.int64)
    n_layers = cfg['num_layers']
    sub = cfg.get('subsample_list') or [False] * n_layers
    n_proj = cfg.get('num_proj', 0) or 0
    concat = cfg.get('subsample_type', 'drop') == 'concat'
    res, dres = bool(cfg.get('residual')), bool(cfg.get('dense_residual'))
    fast = (sum(sub) == 0 and not cfg.get('batch_norm') and n_proj == 0 and not res and
            not dres and capture_layer == 0 and cfg.get('fast', True))   # rnn.py:162
    last_sub = 0                                              # rnn.py:126-132
    for l_rev, s_ in enumerate(sub[::-1]):
        if s_:
            last_sub = n_layers - l_rev
            break
    res_list, captured = [], None
    rnn = cfg.get('rnn_type', 'lstm')                         # rnn.py:162-246 module names
    direction = gru_direction if rnn == 'gru' else lstm_direction
    for l in range(n_layers):
        if fast:   # one multi-layer nn.LSTM / nn.GRU: lstm.weight_ih_l{l}{_reverse}
            names = [prefix + '%s.%s_l%d%s' % (rnn, n, l, s) for s in ('', '_reverse')
                     for n in ('weight_ih', 'weight_hh', 'bias_ih', 'bias_hh')]
        else:      # per-layer modules: lstm_l{l}.weight_ih_l0{_reverse}
            names = [prefix + '%s_l%d.%s_l0%s' % (rnn, l, n, s) for s in ('', '_reverse')
                     for n in ('weight_ih', 'weight_hh', 'bias_ih', 'bias_hh')]
        T_out = int(lens.max())                              # pad_packed -> max len
        xs = xs[:, :T_out]
        fw = direction(xs, lens, *[p[n] for n in names[:4]], reverse=False)
        bw = direction(xs, lens, *[p[n] for n in names[4:]], reverse=True)
        xs = torch.cat([fw, bw], dim=2)
        if capture_layer and l == capture_layer - 1:
            captured = (xs, lens.astype(np.int32))
        if fast or l == n_layers - 1 or not (res or dres or n_proj > 0 or sub[l]):
            continue
        if n_proj > 0:                                        # rnn.py:409-411
            xs = torch.tanh(linear_nd(p, prefix + 'proj_l%d' % l, xs))
        if sub[l]:
            if concat:                                        # rnn.py:421-431
                B_, T_, D_ = xs.shape
                xs = xs[:, :T_ // 2 * 2].reshape(B_, T_ // 2, 2 * D_)
            else:                                             # rnn.py:415-419
                xs = xs[:, 1::2]
            lens = np.full(len(lens), xs.shape[1], np.int64)  # quirk rnn.py:435-439
        elif (res or dres) and l >= last_sub:                 # rnn.py:454-462
            for lower in res_list:
                xs = xs + lower
            res_list = [xs] if res else res_list + [xs]
    if capture_layer:
        return xs, lens.astype(np.int32), perm.astype(np.int64), captured
    return xs, lens.astype(np.int32), perm.astype(np.int64)


def _param_dtype(p):
    """The parameters' float dtype (float64 evaluates the whole restatement in
    double: bench.py's parity reference)."""
    for k, v in p.items():
        if k.endswith('weight') and torch.is_tensor(v):
            return v.dtype
    return torch.float32


def linear_nd(p, name, x):
    """LinearND (linear.py:32-47): affine on the last dim (dropout = 0)."""
    y = torch.matmul(x, p[name + '.fc.weight'].t())
    b = p.get(name + '.fc.bias')
    return y if b is None else y + b


# ---------------------------------------------------------------------------
# CTC (warp-ctc contract, ctc.py:30-66) as an autograd function over float64
# ---------------------------------------------------------------------------
class _CTCOracle(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels_flat, label_lens, act_lens):
        costs, grads = ctc_ref.ctc_batch(logits.detach().numpy(), labels_flat, label_lens,
                                         act_lens, time_major=False)
        ctx.save_for_backward(torch.from_numpy(grads).to(logits.dtype))
        return torch.tensor(costs.sum(), dtype=logits.dtype)

    @staticmethod
    def backward(ctx, g):
        grads, = ctx.saved_tensors
        return grads * g, None, None, None


def ctc_sum(logits, labels_flat, label_lens, act_lens):
    return _CTCOracle.apply(logits, labels_flat, label_lens, act_lens)


def _concat_labels(ys, y_lens):
    """_concatenate_labels (ctc.py:532-549)."""
    return np.concatenate([ys[b, :y_lens[b]] for b in range(len(y_lens))]).astype(np.int64)


def ls_xent(logits, lens, ls_prob, size_average):
    """cross_entropy_label_smoothing (criterion.py:51-80)."""
    B, _, V = logits.shape
    lp = torch.log_softmax(logits, dim=-1)
    tot = sum((-(ls_prob / V) * lp[b, :int(lens[b])]).sum() for b in range(B))
    return tot / B if size_average else tot


def hierarchical_ctc_loss(p, cfg, xs, ys, x_lens, y_lens, ys_sub, y_lens_sub):
    """HierarchicalCTC.forward (hierarchical_ctc.py:267-365): word CTC on the top
    layer, char CTC on the output of layer num_layers_sub (after its dropout,
    before any subsampling, rnn.py:400-407); loss = w_main L_main + w_sub L_sub."""
    xs_t = torch.from_numpy(np.asarray(xs, np.float32)).to(_param_dtype(p))
    top, lens, perm, (mid, lens_sub) = blstm_encoder(p, 'encoder.', dict(cfg, fast=False), xs_t,
                                                     x_lens, capture_layer=cfg['num_layers_sub'])
    B = xs.shape[0]
    terms = []
    for h, ln, head, y, yl in ((top, lens, 'fc_out', ys, y_lens),
                               (mid, lens_sub, 'fc_out_sub', ys_sub, y_lens_sub)):
        logits = linear_nd(p, head, h)
        ys_s = (np.asarray(y) + 1)[perm]
        yl_s = np.asarray(yl)[perm]
        terms.append(ctc_sum(logits, _concat_labels(ys_s, yl_s), yl_s, ln) / B)
    loss_main = terms[0] * cfg['main_loss_weight']
    loss_sub = terms[1] * cfg['sub_loss_weight']
    return loss_main + loss_sub, loss_main, loss_sub


def ctc_model_loss(p, cfg, xs, ys, x_lens, y_lens):
    """CTC.forward (ctc.py:272-342).  xs numpy [B,T,F]; ys numpy [B,L] pad -1."""
    xs_t = torch.from_numpy(np.asarray(xs, np.float32)).to(_param_dtype(p))
    out, out_lens, perm = blstm_encoder(p, 'encoder.', cfg, xs_t, x_lens)
    h = out
    for i in range(len(cfg.get('fc_list', []))):
        h = linear_nd(p, 'fc_%d' % i, h)
    logits = linear_nd(p, 'fc_out', h)
    if cfg.get('logits_temperature', 1) != 1:
        logits = logits / cfg['logits_temperature']
    ys_s = (np.asarray(ys) + 1)[perm]                       # ctc.py:300,310-312
    yl_s = np.asarray(y_lens)[perm]
    B = xs.shape[0]
    loss = ctc_sum(logits, _concat_labels(ys_s, yl_s), yl_s, out_lens) / B
    ls = cfg.get('label_smoothing_prob', 0)
    if ls > 0:
        loss = loss * (1 - ls) + ls_xent(logits, out_lens, ls, False) / B
    return loss, logits, out_lens, perm


# ---------------------------------------------------------------------------
# Location attention (attention_layer.py:74-98, 155-177, 214-251)
# ---------------------------------------------------------------------------
def location_attention(p, prefix, enc_out, enc_out_a, x_lens, dec_out, aw_prev,
                       sharpening=1.0, sigmoid_smoothing=False):
    """enc_out [B,T,E], enc_out_a [B,T,A], dec_out [B,D], aw_prev [B,T].
    Returns ctx [B,E], aw [B,T]."""
    B, T, _ = enc_out.shape
    w = p[prefix + 'conv_head0.weight']                      # [C, 1, 1, K]
    C, K = w.shape[0], w.shape[3]
    f = torch.nn.functional.conv1d(aw_prev.unsqueeze(1), w.view(C, 1, K), padding=K // 2)
    f = f.transpose(1, 2)                                    # [B, T, C]
    pre = (enc_out_a + (dec_out @ p[prefix + 'W_dec_head0.fc.weight'].t()).unsqueeze(1)
           + f @ p[prefix + 'W_conv_head0.fc.weight'].t())
    e = (torch.tanh(pre) @ p[prefix + 'V_head0.fc.weight'].t()).squeeze(2)
    mask = (torch.arange(T).unsqueeze(0) < torch.as_tensor(np.asarray(x_lens)).unsqueeze(1))
    e = e * mask.to(e.dtype)                                 # multiplicative mask :216-225
    e = e * sharpening
    aw = torch.sigmoid(e) if sigmoid_smoothing else torch.softmax(e, dim=-1)
    ctx = (enc_out * aw.unsqueeze(2)).sum(1)
    return ctx, aw


def lstm_cell(p, name, x, h, c):
    """nn.LSTMCell (rnn_decoder.py:48,84-88)."""
    g = (x @ p[name + '.weight_ih'].t() + p[name + '.bias_ih']
         + h @ p[name + '.weight_hh'].t() + p[name + '.bias_hh'])
    H = h.shape[1]
    i, f, gg, o = g.split(H, dim=1)
    c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
    return torch.sigmoid(o) * torch.tanh(c), c


def attention_xe(p, cfg, enc_out, enc_lens, ys, y_lens, perm, task=0, train=None):
    """Teacher-forced decoder of `task` (attention_seq2seq.py:564-607, 704-799):
    bahdanau order, location attention, 1 head, LSTM decoder, forward direction.
    Module names carry the task index (``attend_{task}_fwd`` ...); task 1 is the
    hierarchical model's sub task (hierarchical_attention_seq2seq.py:221-339)
    with num_classes_sub / decoder_num_units_sub.  Returns the XE loss
    (label smoothing included) over the batch, divided by B.

    train (optional): replayed training-mode randomness, all in the sorted
    utterance order -- 'h' [B,S,D] decoder dropout scales on h after the
    LSTMCell (rnn_decoder.py:97-98; the dropped h is dec_out and the state),
    'd' / 'c' [B,S,Dz] scales on the W_d / W_c LinearND outputs (linear.py:45),
    'emb' [B,S,Y] scales on the teacher embeddings, and scheduled sampling
    (attention_seq2seq.py:744-748): 'ss' [S] flags, 'emb_ss' [B,S,Y] scales on
    the sampled embedding embed(argmax logits_{t-1}) (detached).  Test hooks:
    'tok' [B,S] replays given sampled tokens instead of this oracle's argmax,
    '_log' (a list) receives (t, argmax, top-2 gap) of every sampled step."""
    train = train or {}
    B, T, E = enc_out.shape
    ncls = cfg['num_classes'] if task == 0 else cfg['num_classes_sub']
    V = ncls + 1
    eos = ncls
    ys = np.asarray(ys)
    y_lens = np.asarray(y_lens)
    Lp = ys.shape[1]
    ys_in = np.full((B, Lp + 1), eos, np.int64)              # :458-473
    ys_out = np.full((B, Lp + 1), -1, np.int64)
    for b in range(B):
        ys_in[b, 1:y_lens[b] + 1] = ys[b, :y_lens[b]]
        ys_out[b, :y_lens[b]] = ys[b, :y_lens[b]]
        ys_out[b, y_lens[b]] = eos
    ys_in, ys_out, yl = ys_in[perm], ys_out[perm], y_lens[perm]

    D = cfg['decoder_num_units'] if task == 0 else cfg['decoder_num_units_sub']
    sfx = '_%d_fwd' % task
    pre = 'attend%s.' % sfx
    enc_out_a = linear_nd(p, pre + 'W_enc_head0', enc_out)  # :735-739
    init = cfg.get('init_dec_state', 'first')
    c = enc_out.new_zeros(B, D)
    if init == 'zero':
        h = enc_out.new_zeros(B, D)
    else:                                                    # :831-857
        src = {'mean': enc_out.mean(1), 'final': enc_out[:, -1], 'first': enc_out[:, 0]}[init]
        h = torch.tanh(linear_nd(p, 'W_dec_init' + sfx, src))
    dec_out = h
    aw = enc_out.new_zeros(B, T)
    ctx = enc_out.new_zeros(B, E)
    if cfg.get('label_smoothing_prob', 0) > 0:               # Embedding_LS (linear.py:80-116)
        emb_w = p['embed_%d.embed.fc.weight' % task].t()     # [V, emb]
    else:                                                    # Embedding, padding_idx=-1
        emb_w = p['embed_%d.embed.weight' % task]
    ys_emb = emb_w[torch.as_tensor(ys_in)]                   # [B, L+1, emb]
    mk = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in train.items()
          if k not in ('ss', 'tok', '_log')}
    if 'emb' in mk:
        ys_emb = ys_emb * mk['emb']
    ss = train.get('ss')
    logits = []
    for t in range(Lp + 1):                                  # :742-793
        if t > 0:
            if ss is not None and ss[t]:                     # scheduled sampling :744-748
                tok = torch.argmax(logits[-1], dim=-1)
                if '_log' in train:   # test hook: this oracle's argmax and its top-2 gap
                    top2 = torch.topk(logits[-1].detach(), 2, dim=-1).values
                    train['_log'].append((t, tok.clone(), (top2[:, 0] - top2[:, 1]).clone()))
                if 'tok' in train:    # test hook: replay given tokens [B, S]
                    tok = torch.as_tensor(np.asarray(train['tok'])[:, t], dtype=torch.long)
                y = emb_w[tok].detach()
                if 'emb_ss' in mk:
                    y = y * mk['emb_ss'][:, t]
            else:
                y = ys_emb[:, t]
            dec_in = torch.cat([y, ctx], dim=-1)
            h, c = lstm_cell(p, 'decoder%s.lstm_l0' % sfx, dec_in, h, c)
            if 'h' in mk:
                h = h * mk['h'][:, t]
            dec_out = h
        ctx, aw = location_attention(p, pre, enc_out, enc_out_a, enc_lens, dec_out, aw,
                                     cfg.get('sharpening_factor', 1),
                                     cfg.get('sigmoid_smoothing', False))
        a = linear_nd(p, 'W_d' + sfx, dec_out)
        cc = linear_nd(p, 'W_c' + sfx, ctx)
        if 'd' in mk:
            a = a * mk['d'][:, t]
            cc = cc * mk['c'][:, t]
        z = torch.tanh(a + cc)
        logits.append(linear_nd(p, 'fc' + sfx, z))
    logits = torch.stack(logits, 1)                          # [B, L+1, V]
    if cfg.get('logits_temperature', 1) != 1:
        logits = logits / cfg['logits_temperature']
    tgt = torch.as_tensor(ys_out.reshape(-1))
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, V), tgt, ignore_index=-1,
                                             reduction='sum') / B
    ls = cfg.get('label_smoothing_prob', 0)
    if ls > 0:
        loss = loss * (1 - ls) + ls_xent(logits, yl + 1, ls, True)
    return loss


def _enc_cfg(cfg):
    return dict(num_layers=cfg['encoder_num_layers'], subsample_list=cfg['subsample_list'],
                num_proj=cfg.get('encoder_num_proj', 0),
                subsample_type=cfg.get('subsample_type', 'drop'),
                residual=cfg.get('encoder_residual', False),
                dense_residual=cfg.get('encoder_dense_residual', False))


def attention_model_loss(p, cfg, xs, ys, x_lens, y_lens, train=None):
    """AttentionSeq2seq.forward (attention_seq2seq.py:422-562) for the
    bahdanau order, location attention, 1 head, LSTM decoder, forward
    direction only (backward_loss_weight = 0), encoder dropout 0:
    loss = (1 - w_bwd) * XE + lambda * CTC / B.  `train`: see attention_xe."""
    xs_t = torch.from_numpy(np.asarray(xs, np.float32)).to(_param_dtype(p))
    enc_out, enc_lens, perm = blstm_encoder(p, 'encoder.', _enc_cfg(cfg), xs_t, x_lens)
    B = enc_out.shape[0]
    loss = attention_xe(p, cfg, enc_out, enc_lens, ys, y_lens, perm, 0, train)
    loss = loss * (1 - cfg.get('backward_loss_weight', 0))
    lam = cfg.get('ctc_loss_weight', 0)
    if lam > 0:                                              # :534-549, :609-653
        yl = np.asarray(y_lens)[perm]
        lg = linear_nd(p, 'fc_ctc_0', enc_out)
        lab = _concat_labels(np.asarray(ys)[perm] + 1, yl)
        loss = loss + ctc_sum(lg, lab, yl, enc_lens) / B * lam
    return loss


def hierarchical_attention_loss(p, cfg, xs, ys, x_lens, y_lens, ys_sub, y_lens_sub):
    """HierarchicalAttentionSeq2seq.forward (hierarchical_attention_seq2seq.py:
    382-567): word decoder on the top layer, character decoder (task 1) on layer
    encoder_num_layers_sub (after its dropout, before projection / subsampling),
    optional character CTC there.  Returns (loss, loss_main, loss_sub)."""
    xs_t = torch.from_numpy(np.asarray(xs, np.float32)).to(_param_dtype(p))
    top, lens, perm, (mid, lens_sub) = blstm_encoder(
        p, 'encoder.', dict(_enc_cfg(cfg), fast=False), xs_t, x_lens,
        capture_layer=cfg['encoder_num_layers_sub'])
    B = top.shape[0]
    loss_main = attention_xe(p, cfg, top, lens, ys, y_lens, perm, 0) * cfg['main_loss_weight']
    loss = loss_main
    loss_sub = ctc_sub = None
    if cfg['sub_loss_weight'] > 0:
        loss_sub = attention_xe(p, cfg, mid, lens_sub, ys_sub, y_lens_sub, perm, 1) * \
            cfg['sub_loss_weight']
        loss = loss + loss_sub
    w_ctc = cfg.get('ctc_loss_weight_sub', 0)
    if w_ctc > 0:
        yl = np.asarray(y_lens_sub)[perm]
        lg = linear_nd(p, 'fc_ctc_1', mid)
        lab = _concat_labels(np.asarray(ys_sub)[perm] + 1, yl)
        ctc_sub = ctc_sum(lg, lab, yl, lens_sub) / B * w_ctc
        loss = loss + ctc_sub
    return loss, loss_main, (loss_sub if cfg['sub_loss_weight'] > w_ctc else ctc_sub)


def attention_greedy_decode(p, cfg, xs, x_lens, max_len):
    """AttentionSeq2seq.decode(beam_width=1) (attention_seq2seq.py:866-1036):
    bahdanau order, forward decoder, eval mode.  At t = 0 there is no
    recurrence (the <sos> embedding is computed but unused); afterwards the
    input is embed(argmax logits_{t-1}) (torch.max, first maximum); the loop
    stops after the first step at which every utterance emits <eos>.  Returns
    (best_hyps int64 [B, T_out], aw [B, T_out, T], perm) in sorted order."""
    xs_t = torch.from_numpy(np.asarray(xs, np.float32)).to(_param_dtype(p))
    enc_cfg = dict(num_layers=cfg['encoder_num_layers'], subsample_list=cfg['subsample_list'])
    with torch.no_grad():
        enc_out, enc_lens, perm = blstm_encoder(p, 'encoder.', enc_cfg, xs_t, x_lens)
        B, T, E = enc_out.shape
        eos = cfg['num_classes']
        D = cfg['decoder_num_units']
        pre = 'attend_0_fwd.'
        enc_out_a = linear_nd(p, pre + 'W_enc_head0', enc_out)
        init = cfg.get('init_dec_state', 'first')
        c = enc_out.new_zeros(B, D)
        if init == 'zero':
            h = enc_out.new_zeros(B, D)
        else:
            src = {'mean': enc_out.mean(1), 'final': enc_out[:, -1], 'first': enc_out[:, 0]}[init]
            h = torch.tanh(linear_nd(p, 'W_dec_init_0_fwd', src))
        dec_out = h
        aw = enc_out.new_zeros(B, T)
        ctx = enc_out.new_zeros(B, E)
        if cfg.get('label_smoothing_prob', 0) > 0:
            emb_w = p['embed_0.embed.fc.weight'].t()
        else:
            emb_w = p['embed_0.embed.weight']
        tok = torch.full((B,), eos, dtype=torch.long)        # <sos> == <eos> index
        hyps, aws = [], []
        for t in range(max_len):
            if t > 0:
                dec_in = torch.cat([emb_w[tok], ctx], dim=-1)
                h, c = lstm_cell(p, 'decoder_0_fwd.lstm_l0', dec_in, h, c)
                dec_out = h
            ctx, aw = location_attention(p, pre, enc_out, enc_out_a, enc_lens, dec_out, aw,
                                         cfg.get('sharpening_factor', 1),
                                         cfg.get('sigmoid_smoothing', False))
            z = torch.tanh(linear_nd(p, 'W_d_0_fwd', dec_out) + linear_nd(p, 'W_c_0_fwd', ctx))
            logits = linear_nd(p, 'fc_0_fwd', z)
            tok = torch.from_numpy(np.argmax(logits.numpy(), axis=1))   # first maximum
            hyps.append(tok)
            aws.append(aw)
            if bool((tok == eos).all()):
                break
    return (torch.stack(hyps, 1).numpy().astype(np.int64), torch.stack(aws, 1).numpy(),
            perm)


def embedding_padding_row(cfg):
    """nn.Embedding(padding_idx=-1) in linear.py:63-64 zeroes the gradient of
    row num_classes (= <sos>/<eos>); the oracle applies it post-backward."""
    return cfg['num_classes']
