"""Gossiper: relay queue + synchronous model-gossip loop (parity: ``protocols/gossiper.py:31-239``).

Deliberate fixes:

* the relay loop sleeps ``period - elapsed`` (reference sleeps ``period + elapsed``) and wakes
  immediately when a message is queued instead of polling;
* ``gossip_weights`` exits on "status unchanged for X iterations" by comparing *all* recorded
  statuses (reference returns after comparing the first pair);
* the model loop waits for a peer status change (``wait_fn``) or the period — so a round advances
  as soon as peers acknowledge instead of after a fixed ≥1 s sleep.
"""

from __future__ import annotations

import collections
import random
import threading
import time
from typing import Any, Callable, Deque, List, Optional, Tuple

from myfyp_amd.communication.protocols.client import Client
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings
from myfyp_amd.utils.lockcheck import make_lock


class Gossiper(threading.Thread):
    """Relays TTL messages and runs ``gossip_weights`` loops for a node."""

    def __init__(self, self_addr: str, client: Client, period: Optional[float] = None, messages_per_period: Optional[int] = None) -> None:
        super().__init__(daemon=True, name=f"gossiper-thread-{self_addr}")
        self._self_addr = self_addr
        self._client = client
        self.period = Settings.GOSSIP_PERIOD if period is None else period
        self.messages_per_period = Settings.GOSSIP_MESSAGES_PER_PERIOD if messages_per_period is None else messages_per_period
        self._processed: Deque[int] = collections.deque()
        self._processed_set: set = set()
        self._processed_lock = make_lock("Gossiper.processed")
        self._pending: Deque[Tuple[Any, List[str]]] = collections.deque()
        self._cv = threading.Condition()
        self._terminate = threading.Event()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        logger.debug(self._self_addr, "🏁 Starting gossiper...")
        super().start()

    def stop(self) -> None:
        logger.debug(self._self_addr, "🛑 Stopping gossiper...")
        self._terminate.set()
        with self._cv:
            self._cv.notify_all()

    # ------------------------------------------------------------------ relay queue
    def add_message(self, msg: Any, pending_neis: List[str]) -> None:
        if not pending_neis:
            return
        with self._cv:
            self._pending.append((msg, list(pending_neis)))
            self._cv.notify()

    def check_and_set_processed(self, msg_hash: int) -> bool:
        """True the first time a hash is seen (dedup ring of ``AMOUNT_LAST_MESSAGES_SAVED``)."""
        with self._processed_lock:
            if msg_hash in self._processed_set:
                return False
            self._processed.append(msg_hash)
            self._processed_set.add(msg_hash)
            while len(self._processed) > Settings.AMOUNT_LAST_MESSAGES_SAVED:
                self._processed_set.discard(self._processed.popleft())
            return True

    def run(self) -> None:
        while not self._terminate.is_set():
            t0 = time.time()
            batch: List[Tuple[Any, List[str]]] = []
            with self._cv:
                while not self._pending and not self._terminate.is_set():
                    self._cv.wait()
                budget = self.messages_per_period
                while budget > 0 and self._pending:
                    msg, neis = self._pending[0]
                    if len(neis) <= budget:
                        batch.append((msg, neis))
                        self._pending.popleft()
                        budget -= len(neis)
                    else:
                        batch.append((msg, neis[:budget]))
                        self._pending[0] = (msg, neis[budget:])
                        budget = 0
            for msg, neis in batch:
                for nei in neis:
                    self._client.send(nei, msg)
            with self._cv:
                more = bool(self._pending)
            if more and self.period > 0:
                time.sleep(max(0.0, self.period - (time.time() - t0)))

    # ------------------------------------------------------------------ model gossip
    def gossip_weights(
        self,
        early_stopping_fn: Callable[[], bool],
        get_candidates_fn: Callable[[], List[str]],
        status_fn: Callable[[], Any],
        model_fn: Callable[[str], Any],
        period: float,
        create_connection: bool,
        wait_fn: Optional[Callable[[float], None]] = None,
    ) -> None:
        """Synchronous gossip until no candidates remain, early stop, or a stalled status."""
        window = Settings.GOSSIP_EXIT_ON_X_EQUAL_ROUNDS
        last: Deque[str] = collections.deque(maxlen=window)
        while True:
            t0 = time.time()
            if early_stopping_fn():
                logger.info(self._self_addr, "Stopping model gossip process.")
                return
            neis = get_candidates_fn()
            if not neis:
                logger.info(self._self_addr, "🤫 Gossip finished.")
                return
            logger.debug(self._self_addr, f"👥 Gossip remaining nodes: {neis}")
            last.append(str(status_fn()))
            if len(last) == window and len(set(last)) == 1:
                logger.info(self._self_addr, f"⏹️  Gossiping exited for {window} equal rounds.")
                return
            for nei in random.sample(neis, min(Settings.GOSSIP_MODELS_PER_ROUND, len(neis))):
                model = model_fn(nei)
                if model is None:
                    continue
                logger.debug(self._self_addr, f"🗣️ Gossiping model to {nei}.")
                self._client.send(nei, model, create_connection=create_connection)
            remaining = max(0.0, period - (time.time() - t0))
            if wait_fn is not None:
                wait_fn(remaining)
            elif remaining > 0:
                time.sleep(remaining)
