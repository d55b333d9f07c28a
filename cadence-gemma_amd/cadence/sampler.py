"""Greedy / categorical sampler for the MI355X Griffin.

Keeps the API of the reference `recurrentgemma/torch/sampler.py`
(`SamplingState` :33-53, `SamplerOutput` :56-67, `Sampler(model, vocab,
greedy_sampling, is_it_model)` :70-109, `__call__(input_strings,
total_generation_steps, echo, return_logits, end_sampling_at_eos_token,
img_path)` :377-449) with the position semantics of the working multimodal
sampler `examples/cadence_sampler.py` (:185-298): left-padded prompts,
positions `arange(T) - T + len` clipped at -1, prefill on tokens[:, :-1]
(image spliced there), one cached step on the last prompt token, then
single-token decode.  The library's `prompt_length += 729` /
`input_lengths + 1` bugs are not reproduced.

Decode runs on device: soft-cap + argmax are fused into the logits kernel,
the next token / positions / step counter are advanced by a kernel, and the
whole step can be captured once into a hipGraph and replayed
(`use_graph=True`), so the loop has no per-step host sync.

EOS stopping (`end_sampling_at_eos_token=True`) keeps the reference's
behaviour by default (recurrentgemma/torch/sampler.py:177-187, 209-225):
`done_now = torch.equal(next_token, eos)` compares the batch's [B] tokens
with a [1] tensor, so only a batch of ONE row ever stops -- after a decode
step samples EOS (the token sampled from the prompt is never tested), the
rest of the buffer stays pad -- and rows of a larger batch keep generating
after their EOS.  `eos_per_row=True` opts into per-row stopping instead:
each row is padded after its first EOS (the first token included) and the
loop ends once every row is done.
"""

from __future__ import annotations

import dataclasses
from typing import Generic, NamedTuple, Sequence, TypeVar

import os

import torch

from . import common, ops
from .tracing import trace
from .modules import AttentionBlockCache

Cache = TypeVar("Cache")


@dataclasses.dataclass
class SamplingState(Generic[Cache]):
  tokens_buffer: torch.Tensor
  step: torch.Tensor
  total_steps: torch.Tensor
  positions: torch.Tensor
  cache: Cache
  done: torch.Tensor
  logits_buffer: torch.Tensor | None = None


class SamplerOutput(NamedTuple):
  text: list[str]
  logits: list[torch.Tensor]
  tokens: list[torch.Tensor]


def _to_device(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
  """A host tensor on `dev` without blocking the host (pinned staging; the
  caching host allocator keeps the block until the copy has run)."""
  if dev.type != "cuda" or t.is_cuda or os.environ.get("CADENCE_SYNC_H2D") == "1":
    return t.to(dev)        # (the env switch: lab A/B of the blocking copy)
  return t.pin_memory().to(dev, non_blocking=True)


def prompt_positions(lengths: torch.Tensor, prompt_length: int) -> torch.Tensor:
  """examples/cadence_sampler.py:198-201."""
  pos = torch.arange(prompt_length, dtype=torch.int32)[None].repeat(
      lengths.shape[0], 1)
  pos = pos - prompt_length + lengths.to(torch.int32)[:, None]
  return torch.clip(pos, min=-1)


class Sampler:
  """Sampler for a `cadence.Griffin` model."""

  def __init__(self, model, vocab, greedy_sampling: bool = True,
               is_it_model: bool = False, use_graph: bool = True,
               eos_per_row: bool = False):
    self.model = model
    self.vocab = vocab
    self.greedy_sampling = greedy_sampling
    self._is_it_model = is_it_model
    self.use_graph = use_graph
    self.eos_per_row = eos_per_row
    self._eos_token = torch.tensor([self.vocab.eos_id()], device=self.device)

  @property
  def dtype(self) -> torch.dtype:
    return next(self.model.parameters()).dtype

  @property
  def device(self) -> torch.device:
    return next(self.model.parameters()).device

  @property
  def vocab_size(self) -> int:
    return self.model.config.vocab_size

  def apply_model(self, tokens, segment_pos, cache=None, return_logits=True,
                  return_cache=True, img_path=None, images=None,
                  image_splice=None):
    return self.model(tokens=tokens, segment_pos=segment_pos, cache=cache,
                      return_logits=return_logits, return_cache=return_cache,
                      img_path=img_path, images=images,
                      image_splice=image_splice)

  def tokenize(self, input_string: str) -> torch.Tensor:
    if self._is_it_model:
      input_string = common.apply_it_formatter(input_string)
    ids = [self.vocab.bos_id()] + list(self.vocab.EncodeAsIds(input_string))
    return torch.tensor(ids, dtype=torch.int32)

  def _get_padded_tokens(self, tokens: Sequence[torch.Tensor]) -> torch.Tensor:
    n = max(len(t) for t in tokens)
    rows = [torch.cat([torch.full([n - len(t)], self.vocab.pad_id(),
                                  dtype=torch.int32), t]) for t in tokens]
    return torch.stack(rows)

  # ------------------------------------------------------------ generation

  @torch.no_grad()
  def generate(self, tokens: torch.Tensor, input_lengths: torch.Tensor,
               total_generation_steps: int, images=None, img_path=None,
               return_logits: bool = False, echo: bool = False,
               end_sampling_at_eos_token: bool = False,
               events: dict | None = None, slot: int = 0) -> SamplingState:
    """Prefill + decode for a left-padded [B, T] prompt batch (on device).

    `events`, if given, receives HIP events bracketing the prefill
    ("prefill_start"/"prefill_end") and the graph-replayed decode steps
    ("decode_start"/"decode_end", with "decode_steps").  Everything runs
    on the caller's current stream (the decode graph is replayed there);
    `slot` picks the decode graph (static buffers) -- calls that may overlap
    on different streams must use different slots (`generate_many`).
    """
    dev = self.device
    b, t = tokens.shape
    if not tokens.is_cuda and tokens.numel():
      # nn.Embedding raises on an id outside [0, V) (modules.py:994-1001);
      # the embedding kernel cannot, so host-side prompts are checked here
      lo, hi = int(tokens.min()), int(tokens.max())
      if lo < 0 or hi >= self.vocab_size:
        raise ValueError(f"prompt token ids must lie in [0, {self.vocab_size}); "
                         f"got [{lo}, {hi}]")
    pos_cpu = prompt_positions(input_lengths.cpu(), t)
    # host -> device through pinned memory, asynchronous: a pageable copy
    # blocks the host until the stream has drained, so with two lanes the
    # host could not enqueue micro-batch j + 2 before j had finished
    positions = _to_device(pos_cpu, dev)
    # image tokens spliced in front by the prefill (griffin.py:179: only when
    # the prompt holds a position 0); known on the host, so the decode graph
    # copies only the attention-cache slots the prefill wrote
    n_img = 0
    model_vis = getattr(self.model, "vision_config", None)
    splice_all = bool((pos_cpu == 0).any())     # the whole prompt in one call
    splice = bool((pos_cpu[:, :-1] == 0).any()) if t > 1 else splice_all
    if (images is not None or img_path) and model_vis is not None and splice:
      n_img = self.model.n_visual_tokens
    tokens = (tokens.to(dev, torch.int32) if tokens.is_cuda else
              _to_device(tokens.to(torch.int32), dev))
    steps = total_generation_steps
    # the reference's torch.equal(next_token, eos) only ever holds for B == 1
    eos_stop = end_sampling_at_eos_token and (self.eos_per_row or b == 1)
    if steps == 0:
      prev_logits, _ = self.apply_model(tokens, positions, None,
                                        return_logits and echo, False,
                                        img_path, images, splice_all)
      buf = tokens if echo else torch.empty(b, 0, dtype=torch.int32, device=dev)
      lb = prev_logits[:, -t:] if (return_logits and echo) else None
      return SamplingState(buf, torch.tensor(0), torch.tensor(0), positions,
                           None, torch.zeros(b, dtype=torch.bool), lb)
    model = self.model
    prev_logits = None
    if events is not None:
      events["prefill_start"] = torch.cuda.Event(enable_timing=True)
      events["prefill_end"] = torch.cuda.Event(enable_timing=True)
      events["prefill_start"].record()
    # greedy, no logits: the last prompt token's cached step is the first
    # replay of the decode graph (no eager ~200-launch step)
    graph_first = (t > 1 and self.use_graph and self.greedy_sampling and
                   not return_logits and steps > 2)
    if t > 1:
      with trace("sampler:prefill"):
        prev_logits, cache = self.apply_model(tokens[:, :-1], positions[:, :-1],
                                              None, return_logits and echo, True,
                                              img_path, images, splice)
      if events is not None:
        events["prefill_end"].record()
      if graph_first:
        buf = torch.full((b, steps), self.vocab.pad_id(), dtype=torch.int32,
                         device=dev)
        pos = positions[:, -1].to(torch.int32).contiguous()
        step = torch.zeros(1, dtype=torch.int32, device=dev)
        cur = tokens[:, -1].to(torch.int32).contiguous()
        done = self._decode_graph(cur, pos, cache, buf, step, steps,
                                  eos_stop, events, start=0,
                                  cache_len=n_img + t - 1, slot=slot)
        if echo:
          buf = torch.cat([tokens, buf], dim=1)
        return SamplingState(buf, step, torch.tensor(steps), pos[:, None], cache,
                             done, None)
      nxt, logits, cache = model.next_token(tokens[:, -1:], positions[:, -1:],
                                            cache, return_logits or
                                            not self.greedy_sampling)
    else:
      logits_all, cache = self.apply_model(tokens, positions, None, True, True,
                                           img_path, images, splice_all)
      logits = logits_all[:, -1]
      nxt = self._sample(logits)
    if not self.greedy_sampling:
      nxt = self._sample(logits)
    first_logits = logits
    buf = torch.full((b, steps), self.vocab.pad_id(), dtype=torch.int32,
                     device=dev)
    lbuf = None
    if return_logits:
      lbuf = torch.zeros(b, steps, self.vocab_size, dtype=self.dtype,
                         device=dev)
      lbuf[:, 0] = logits
    # the first token goes through the same on-device bookkeeping as the
    # rest: buf[:, 0], positions + 1, step 1, EOS flags
    pos = positions[:, -1].to(torch.int32).contiguous()
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    cur = torch.empty(b, dtype=torch.int32, device=dev)
    dflags = self._done_flags(b, eos_stop)
    self._advance(nxt, buf, step, pos, cur, dflags)
    n_more = steps - 1
    graphable = (self.use_graph and self.greedy_sampling and not return_logits
                 and n_more > 1)
    if graphable:
      done = self._decode_graph(cur, pos, cache, buf, step, n_more,
                                eos_stop, events,
                                cache_len=n_img + t, done_in=dflags, slot=slot)
    else:
      watch = _DoneWatch(dflags)
      for i in range(n_more):
        if watch.finished(i):
          break
        nxt, logits, cache = model.next_token(cur[:, None], pos[:, None], cache,
                                              return_logits or not
                                              self.greedy_sampling)
        if not self.greedy_sampling:
          nxt = self._sample(logits)
        if return_logits:
          lbuf[:, i + 1] = logits
        self._advance(nxt, buf, step, pos, cur, dflags)
      done = _row_done(dflags, b, dev)
    if echo:
      buf = torch.cat([tokens, buf], dim=1)
      if return_logits:
        # examples/cadence_sampler.py:283: [prev_logits, logits, buffer] -- the
        # last prompt position's logits appear twice (also buffer[:, 0]).
        prompt_logits = prev_logits[:, -(t - 1):] if t > 1 else lbuf[:, :0]
        lbuf = torch.cat([prompt_logits, first_logits[:, None].to(lbuf.dtype),
                          lbuf], dim=1)
    return SamplingState(buf, step, torch.tensor(steps), pos[:, None], cache,
                         done, lbuf)

  @torch.no_grad()
  def generate_many(self, batches: Sequence[tuple], total_generation_steps: int,
                    lanes: int = 2, events: dict | None = None,
                    continuous: bool = False) -> list[SamplingState]:
    """Generation for a sequence of micro-batches, pipelined over `lanes`
    streams: micro-batch j runs whole (prefill, then its decode graph
    replays) on one lane, the lanes taken in turn, so one lane's prefill
    (MFMA-bound GEMMs, plus the vision tower's side stream) overlaps another
    lane's decode steps (a latency-bound GEMV chain) on the GPU.  Each lane
    has its own decode graph (static buffers, arrival counters).  `batches`:
    (tokens [B, T], input_lengths [B], images or None) per micro-batch; the
    outputs equal `generate` on each in turn.  `events` applies to the last
    micro-batch.

    Default: the lanes start after the caller's stream and the caller's
    stream waits for them at return (the states are ready on it).
    `continuous`: a serving loop's form -- the lanes wait only for the
    caller's stream as it is at this call (the inputs), the turn of lanes
    carries on from the previous continuous call, and nothing joins back:
    the next call's first prefill overlaps this call's last decode.  Hand
    the states to a consumer stream with `hand_over`."""
    dev = self.device
    cur = torch.cuda.current_stream(dev)
    ls = self.__dict__.setdefault("_lanes", {})
    streams = ls.setdefault(dev, [])
    while len(streams) < lanes:
      streams.append(torch.cuda.Stream(device=dev))
    streams = streams[:lanes]
    if continuous:
      inputs = torch.cuda.Event()
      inputs.record(cur)
      first = self.__dict__.get("_lane_next", 0) % lanes
    else:
      first = 0
    used = []
    for s in streams:
      if continuous:
        s.wait_event(inputs)
      else:
        s.wait_stream(cur)
    states = []
    for j, (tokens, lengths, images) in enumerate(batches):
      lane = (first + j) % lanes
      ev = events if j == len(batches) - 1 else None
      if lane not in used:
        used.append(lane)
      with torch.cuda.stream(streams[lane]):
        # lanes own decode graphs 1..lanes: a plain generate() (slot 0, the
        # caller's stream) right after a continuous call, whose lanes are
        # still replaying, never shares a graph's static buffers with them
        states.append(self.generate(tokens, lengths, total_generation_steps,
                                    images=images, events=ev, slot=1 + lane))
    if continuous:
      self._lane_next = (first + len(batches)) % lanes
      self._ready = []
      for lane in used:
        e = torch.cuda.Event()
        e.record(streams[lane])
        self._ready.append(e)
      return states
    for s in streams:
      cur.wait_stream(s)
    self._record(states, cur)
    return states

  def hand_over(self, states: Sequence[SamplingState], stream) -> None:
    """Makes `stream` wait for the lanes of the last continuous
    `generate_many` and hands the states' memory to it."""
    for e in getattr(self, "_ready", ()):
      stream.wait_event(e)
    self._record(states, stream)

  @staticmethod
  def _record(states, stream):
    for st in states:   # allocated on a lane stream, used on `stream`
      for t in (st.tokens_buffer, st.step, st.positions, st.done):
        if isinstance(t, torch.Tensor) and t.is_cuda:
          t.record_stream(stream)
      for v in (st.cache or {}).values():
        for t in v:
          t.record_stream(stream)

  def _sample(self, logits: torch.Tensor) -> torch.Tensor:
    if self.greedy_sampling:
      return torch.argmax(logits, dim=-1).to(torch.int32)
    return torch.distributions.Categorical(logits=logits.float()).sample().to(
        torch.int32)

  def _done_flags(self, b, eos_stop):
    """int32[B + 1] on-device EOS flags (row latches, all-rows flag), or None
    when sampling does not stop at EOS."""
    if not eos_stop:
      return None
    return torch.zeros(b + 1, dtype=torch.int32, device=self.device)

  def _eos_args(self):
    """(eos_id, pad_id, eos_from) of decode_advance: the reference never
    tests the first token (column 0); per-row stopping does."""
    return (int(self.vocab.eos_id()), int(self.vocab.pad_id()),
            0 if self.eos_per_row else 1)

  def _advance(self, nxt, buf, step, pos, cur, dflags):
    ops.ops.decode_advance_(nxt, buf, step, pos, cur, dflags, *self._eos_args())

  def _decode_graph(self, cur, pos, cache, buf, step, n_more, eos_stop,
                    events=None, start=1, cache_len=None, done_in=None, slot=0):
    """Replays a captured single-token decode step `n_more` times.

    The graph holds raw pointers to the model's (packed) weights, so it is
    keyed on the parameters' storage and version counters: a weight reload
    or in-place update recaptures it.  One graph per `slot` (its own static
    buffers and capture stream, hence its own arrival counters)."""
    if not hasattr(self, "_graphs"):
      self._graphs = {}
    key = (cur.shape[0], cur.device, bool(eos_stop), slot)
    version = tuple((p.data_ptr(), p._version) for p in self.model.parameters())
    eng = self._graphs.get(key)
    if eng is None or eng.max_steps < buf.shape[1] or eng.version != version:
      self._graphs.pop(key, None)
      eng = _DecodeGraph(self.model, cache, cur.shape[0], buf.shape[1],
                         cur.device, eos_stop, self._eos_args())
      eng.version = version
      self._graphs[key] = eng
    return eng.run(cache, cur, pos, buf, step, n_more, events, start,
                   cache_len, done_in)

  # ------------------------------------------------------------------- API

  @torch.no_grad()
  def __call__(self, input_strings: Sequence[str], total_generation_steps: int,
               echo: bool = False, return_logits: bool = False,
               end_sampling_at_eos_token: bool = True,
               img_path: str | None = None,
               images: torch.Tensor | None = None) -> SamplerOutput:
    if total_generation_steps < 0:
      raise ValueError("total_generation_steps must be at least 0.")
    ids = [self.tokenize(s) for s in input_strings]
    lengths = torch.tensor([len(x) for x in ids], dtype=torch.int32)
    padded = self._get_padded_tokens(ids)
    pad_lengths = padded.shape[1] - lengths
    state = self.generate(padded, lengths, total_generation_steps, images,
                          img_path, return_logits, echo,
                          end_sampling_at_eos_token)
    toks = [row[int(l):].cpu() for row, l in zip(state.tokens_buffer,
                                                  pad_lengths)]
    logits = []
    if return_logits:
      logits = [row[int(l):] for row, l in zip(state.logits_buffer,
                                               pad_lengths)]
    return SamplerOutput(
        text=[self.vocab.DecodeIds(t.tolist()) for t in toks],
        logits=logits, tokens=toks)


def _clone_cache(cache):
  return {k: type(v)(*[t.clone() for t in v]) for k, v in cache.items()}


def _row_done(dflags, b, dev):
  if dflags is None:
    return torch.zeros(b, dtype=torch.bool, device=dev)
  return dflags[:b].bool()


class _DoneWatch:
  """Host view of the on-device all-rows-done flag without stalling the GPU.

  Every `every` steps the flag is copied (async) into pinned memory behind
  an event; the check waits only on the copy issued one period earlier, so
  the host stays at most two periods ahead of the GPU and the GPU queue
  never drains.  Steps issued after the rows finished only write pad
  (decode_advance latches per row), so stopping late changes no output.
  """

  def __init__(self, dflags, every=8):
    self.flags = dflags
    self.every = every
    self.pending = []
    if dflags is not None:
      self.host = torch.zeros(2, dtype=torch.int32, pin_memory=True)

  def finished(self, i):
    if self.flags is None or i == 0 or i % self.every:
      return False
    slot = (i // self.every) % 2
    ev = torch.cuda.Event()
    self.host[slot:slot + 1].copy_(self.flags[-1:], non_blocking=True)
    ev.record()
    self.pending.append((slot, ev))
    if len(self.pending) < 2:
      return False
    pslot, pev = self.pending.pop(0)
    pev.synchronize()
    return bool(self.host[pslot])


class _DecodeGraph:
  """One single-token decode step captured into a hipGraph.

  Static buffers: current token, positions, token buffer, step counter, the
  EOS flags and a private copy of every block cache (recurrent states and
  attention ring buffers are updated in place by the kernels); for B <= 32
  also the step's input rows (row-major and packed), which each replay's
  tail launch fills for the next one, and that launch's arrival counter.  `run`
  copies the prefill state in, replays the graph, and copies the generated
  tokens out, all on the caller's current stream.  Capture happens on a
  private stream (hipGraph capture cannot use the null stream), which also
  keys the graph's own arrival counters.
  """

  def __init__(self, model, cache_like, batch, max_steps, device, eos_stop,
               eos_args):
    self.model = model
    self.max_steps = max_steps
    self.eos_args = eos_args
    self.cur = torch.zeros(batch, dtype=torch.int32, device=device)
    self.pos = torch.zeros(batch, dtype=torch.int32, device=device)
    self.buf = torch.zeros(batch, max_steps, dtype=torch.int32, device=device)
    self.step = torch.ones(1, dtype=torch.int32, device=device)
    self.done = (torch.zeros(batch + 1, dtype=torch.int32, device=device)
                 if eos_stop else None)
    # the step's input rows, written by the previous replay's tail (the first
    # replay's by `run`), and the tail's arrival counter
    self.chained = ops.want_packed(batch, model.config.width)
    if self.chained:
      self.x = torch.zeros(batch, model.config.width, dtype=model.embedder.input_embedding.dtype,
                           device=device)
      self.xp = ops.packed_empty(batch, model.config.width, device).zero_()
      self.counter = torch.zeros(1, dtype=torch.int32, device=device)
    self.cache = _clone_cache(cache_like)
    self.stream = torch.cuda.Stream(device=device)
    self.stream.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(self.stream):
      self._step()                     # warm-up (allocator pools, packing)
      self.graph = torch.cuda.CUDAGraph()
      with torch.cuda.graph(self.graph, stream=self.stream):
        self._step()
    torch.cuda.current_stream(device).wait_stream(self.stream)
    ops.claim_counters(self.stream, self)

  def _step(self):
    if self.chained:
      # (input rows already embedded) blocks -> logits -> one tail launch:
      # argmax, bookkeeping, the next step's embedding
      # (Griffin.next_token_chained)
      self.model.next_token_chained(
          self.x, self.xp, self.pos, self.cache,
          dict(buf=self.buf, step=self.step, pos=self.pos, cur=self.cur, done=self.done,
               eos_args=self.eos_args, counter=self.counter))
      return
    nxt, _, _ = self.model.next_token(self.cur[:, None], self.pos[:, None],
                                      self.cache, False, inplace=True)
    ops.ops.decode_advance_(nxt, self.buf, self.step, self.pos, self.cur,
                            self.done, *self.eos_args)

  @staticmethod
  def _copy_cache(dst_cache, src_cache, slots):
    """Copies block caches; of the attention ring buffers only the first
    `slots` slots (the ones written so far; decode attention never reads a
    slot at or past num_tokens before the ring wraps), all when None:
    the (dst, src) pairs, for one ops.copy_batched_ with the other
    hand-over copies."""
    return [(d[:, :slots], s_[:, :slots])
            if (isinstance(src, AttentionBlockCache) and slots is not None and
                d.dim() == 4 and slots < d.shape[1]) else (d, s_)
            for name, src in src_cache.items()
            for d, s_ in zip(dst_cache[name], src)]

  def run(self, cache, cur, pos, buf, step, n_more, events=None, start=1,
          cache_len=None, done_in=None):
    """Replays the step `n_more` times from buffer column `start` (the
    tokens before it are already in `buf`, the rest of `buf` is pad).
    `cache_len`: tokens already in the attention caches (host-known), so
    only written ring slots move.  Returns the per-row done flags."""
    steps = buf.shape[1]
    # the prefill state in: cache, token, position, buffer (no columns left
    # from an earlier run), flags -- one batched copy launch
    pairs = self._copy_cache(self.cache, cache, cache_len)
    pairs += [(self.cur, cur), (self.pos, pos), (self.buf[:, :steps], buf)]
    if self.done is not None and done_in is not None:
      pairs.append((self.done, done_in))
    ops.copy_batched_(pairs)
    if self.chained:
      # the first replay's input rows (later replays' come from the tail)
      self.model.embedder.encode_packed_into(self.cur, self.x, self.xp)
    self.step.fill_(start)
    if self.done is not None and done_in is None:
      self.done.zero_()
    watch = _DoneWatch(self.done)
    if events is not None:   # the replays alone (cache copies excluded)
      events["decode_start"] = torch.cuda.Event(enable_timing=True)
      events["decode_end"] = torch.cuda.Event(enable_timing=True)
      events["decode_steps"] = n_more
      events["decode_start"].record()
    done = 0
    with trace("sampler:decode"):
      for i in range(n_more):
        if watch.finished(i):
          break
        self.graph.replay()
        done += 1
    if events is not None:
      events["decode_end"].record()
    pairs = [(buf[:, start:], self.buf[:, start:steps]), (step, self.step),
             (pos, self.pos), (cur, self.cur)]
    pairs += self._copy_cache(cache, self.cache,
                              None if cache_len is None else cache_len + done)
    ops.copy_batched_(pairs)
    return _row_done(self.done, cur.shape[0], cur.device).clone()
