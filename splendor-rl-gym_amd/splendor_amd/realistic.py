"""Realistic multi-player mode: host mirror of the reference's types (src/solver.py:25-200, 471-860).

``GameConfig``, ``GemPool``, ``CardMarket``, ``PlayerState`` and ``MultiPlayerState`` keep the
reference's fields, constructors, hashing and printing; ``MultiPlayerState.solve`` runs the beam
search on the MI355X engine (``sbr_*`` entry points of libsplendor_beam.so; 2-4 players, the gem
pool limited (the CLI's and config C4's case) or unlimited (``infinite_resources=True``, whose takes
are the speedrun take table, src/solver.py:635-659)).  Packed device form: 12 x u64 per state
(``include/splendor_beam.h``).
"""
from __future__ import annotations

import random
from dataclasses import dataclass

import numpy as np

from .codec import decode as _dec_player
from .codec import encode as _enc_player
from .deck import COLOR_NUM, get_deck

deck = get_deck()
RW = 12


@dataclass(frozen=True)
class GameConfig:
    """Rules of a game (src/solver.py:25-33)."""

    num_players: int = 2
    target_points: int = 15
    gems_per_color: int = 4
    cards_visible_per_tier: int = 4
    infinite_resources: bool = True


@dataclass(frozen=True)
class GemPool:
    """Global gem pool (src/solver.py:36-80)."""

    available: tuple

    @classmethod
    def new_pool(cls, gems_per_color: int) -> 'GemPool':
        return cls(available=tuple(gems_per_color for _ in range(COLOR_NUM)))

    def can_take_three_different(self, gems_requested) -> bool:
        if sum(1 for g in gems_requested if g > 0) != 3:
            return False
        return all(gems_requested[i] <= 1 and self.available[i] >= gems_requested[i] for i in range(COLOR_NUM))

    def can_take_two_same(self, gems_requested) -> bool:
        if sum(gems_requested) != 2:
            return False
        idx = next((i for i in range(COLOR_NUM) if gems_requested[i] == 2), None)
        return idx is not None and self.available[idx] >= 4

    def take(self, gems) -> 'GemPool':
        return GemPool(tuple(self.available[i] - gems[i] for i in range(COLOR_NUM)))

    def return_gems(self, gems) -> 'GemPool':
        return GemPool(tuple(self.available[i] + gems[i] for i in range(COLOR_NUM)))


def tier_lists(shuffle: bool = False, seed=None):
    """Tier card orders: pt 0 / pt 1-2 / pt >= 3, shuffled by random.Random(seed) (src/solver.py:94-119)."""
    t1 = [i for i, c in enumerate(deck) if c.pt == 0]
    t2 = [i for i, c in enumerate(deck) if c.pt in (1, 2)]
    t3 = [i for i, c in enumerate(deck) if c.pt >= 3]
    if shuffle:
        rng = random.Random(seed)
        rng.shuffle(t1)
        rng.shuffle(t2)
        rng.shuffle(t3)
    return t1, t2, t3


@dataclass(frozen=True)
class CardMarket:
    """Visible cards and decks (src/solver.py:83-174)."""

    tier1_visible: tuple
    tier2_visible: tuple
    tier3_visible: tuple
    tier1_deck: tuple
    tier2_deck: tuple
    tier3_deck: tuple

    @classmethod
    def from_full_deck(cls, shuffle: bool = False, seed=None) -> 'CardMarket':
        t1, t2, t3 = tier_lists(shuffle, seed)
        return cls(tuple(t1[:4]), tuple(t2[:4]), tuple(t3[:4]), tuple(t1[4:]), tuple(t2[4:]), tuple(t3[4:]))

    def _tiers(self):
        return [(self.tier1_visible, self.tier1_deck), (self.tier2_visible, self.tier2_deck),
                (self.tier3_visible, self.tier3_deck)]

    def buy_card(self, card_idx: int) -> 'CardMarket':
        tiers = self._tiers()
        for t, (vis, dk) in enumerate(tiers):
            if card_idx in vis:
                v = list(vis)
                v.remove(card_idx)
                if dk:
                    v.append(dk[0])
                    dk = dk[1:]
                tiers[t] = (tuple(v), dk)
                return CardMarket(tiers[0][0], tiers[1][0], tiers[2][0], tiers[0][1], tiers[1][1], tiers[2][1])
        return self

    def all_visible_cards(self) -> tuple:
        return self.tier1_visible + self.tier2_visible + self.tier3_visible


@dataclass(frozen=True)
class PlayerState:
    """One player (src/solver.py:177-200)."""

    player_id: int
    cards: tuple
    bonus: tuple
    gems: tuple
    pts: int
    saved: int

    def total_gem_count(self) -> int:
        return sum(self.gems)

    def can_afford(self, card_idx: int) -> bool:
        card = deck[card_idx]
        return all(self.gems[i] + self.bonus[i] >= card.cost[i] for i in range(COLOR_NUM))


class MultiPlayerState:
    """Complete realistic game state (src/solver.py:471-566)."""

    def __init__(self, config, players, gem_pool, market, current_player, turn_number,
                 final_round_triggered=False, final_round_player=None):
        self.config = config
        self.players = players
        self.gem_pool = gem_pool
        self.market = market
        self.current_player = current_player
        self.turn_number = turn_number
        self.final_round_triggered = final_round_triggered
        self.final_round_player = final_round_player
        self.hash = hash((self.players, self.gem_pool.available, self.market.all_visible_cards(), self.current_player))

    @classmethod
    def newgame(cls, config: GameConfig | None = None, shuffle_market: bool = False, seed=None) -> 'MultiPlayerState':
        if config is None:
            config = GameConfig(infinite_resources=False)
        no_gems = (0,) * COLOR_NUM
        players = tuple(PlayerState(i, (), no_gems, no_gems, 0, 0) for i in range(config.num_players))
        return cls(config, players, GemPool.new_pool(config.gems_per_color),
                   CardMarket.from_full_deck(shuffle_market, seed), 0, 0)

    def __repr__(self):
        cur = self.players[self.current_player]
        return f'Turn {self.turn_number}, P{self.current_player}: {cur.pts}pts, {cur.gems!r}'

    def __hash__(self):
        return self.hash

    def __eq__(self, other) -> bool:
        return self.hash == other.hash

    def is_game_over(self) -> bool:
        if not self.final_round_triggered:
            return any(p.pts >= self.config.target_points for p in self.players)
        return self.current_player == self.final_round_player

    def get_winner(self):
        if not self.is_game_over():
            return None
        mx = max(p.pts for p in self.players)
        w = [p for p in self.players if p.pts == mx]
        if len(w) == 1:
            return w[0].player_id
        mc = min(len(p.cards) for p in w)
        w = [p for p in w if len(p.cards) == mc]
        return w[0].player_id if len(w) == 1 else None

    # ------------------------------------------------------------ packed form
    def tiers(self):
        """Full tier orders (visible + deck) of the game's original market, needed by the device."""
        return self._tiers0

    def pack(self, tiers0) -> np.ndarray:
        return pack_state(self, tiers0)

    def solve(self, *, use_heuristic: bool = True, heuristic_name: str = 'competitive', beam_width: int = 20_000,
              verbose: bool = True, device: int = 0, tiers=None, sync_random: bool = True):
        """Beam search to game over on the MI355X engine (src/solver.py:750-860)."""
        from .engine_rt import solve_realistic
        return solve_realistic(self, beam_width=beam_width, verbose=verbose, device=device, tiers=tiers,
                               heuristic_name=heuristic_name, sync_random=sync_random)


def pack_state(s: MultiPlayerState, tiers0) -> np.ndarray:
    """12-word packed form (oracle/csrc/oracle.c, realistic section)."""
    w = np.zeros(RW, dtype=np.uint64)
    for i, p in enumerate(s.players):
        lo, hi = _enc_player(p.cards, p.gems, p.pts, p.saved)
        w[2 * i], w[2 * i + 1] = lo, hi
    m = 0
    if s.config.infinite_resources:   # the pool grows by the gems paid: 12-bit fields in w[11]
        if any(v < 0 or v > 4095 for v in s.gem_pool.available):
            raise ValueError('gem pool outside the packed range')
        w[11] = sum(v << (12 * c) for c, v in enumerate(s.gem_pool.available))
    else:
        for c, v in enumerate(s.gem_pool.available):
            m |= v << (3 * c)
    m |= s.current_player << 15
    m |= (1 if s.final_round_triggered else 0) << 17
    m |= (7 if s.final_round_player is None else s.final_round_player) << 18
    vis = [s.market.tier1_visible, s.market.tier2_visible, s.market.tier3_visible]
    decks = [s.market.tier1_deck, s.market.tier2_deck, s.market.tier3_deck]
    for t in range(3):
        m |= (len(tiers0[t]) - 4 - len(decks[t])) << (21 + 6 * t)
        m |= len(vis[t]) << (39 + 3 * t)
    w[8] = m
    v0 = v1 = 0
    for t in range(3):
        for j, c in enumerate(vis[t]):
            if t == 0:
                v0 |= c << (7 * j)
            elif t == 1:
                v0 |= c << (28 + 7 * j)
            else:
                v1 |= c << (7 * j)
    w[9], w[10] = v0, v1
    return w


def unpack_state(w, config: GameConfig, tiers0, turn_number: int) -> MultiPlayerState:
    w = [int(x) for x in w]
    players = []
    for i in range(config.num_players):
        cards, bonus, gems, pts, saved = _dec_player(w[2 * i], w[2 * i + 1])
        players.append(PlayerState(i, cards, bonus, gems, pts, saved))
    m = w[8]
    if config.infinite_resources:
        pool = tuple((w[11] >> (12 * c)) & 4095 for c in range(5))
    else:
        pool = tuple((m >> (3 * c)) & 7 for c in range(5))
    cp = (m >> 15) & 3
    frt = bool((m >> 17) & 1)
    frp = (m >> 18) & 7
    vis, decks = [], []
    for t in range(3):
        dptr = (m >> (21 + 6 * t)) & 63
        nv = (m >> (39 + 3 * t)) & 7
        word = (w[9] >> (28 * t)) if t < 2 else w[10]
        vis.append(tuple((word >> (7 * j)) & 127 for j in range(nv)))
        decks.append(tuple(tiers0[t][4 + dptr:]))
    market = CardMarket(vis[0], vis[1], vis[2], decks[0], decks[1], decks[2])
    return MultiPlayerState(config, tuple(players), GemPool(pool), market, cp, turn_number, frt,
                            None if frp == 7 else frp)


def game_params(config: GameConfig, tiers0) -> tuple[np.ndarray, np.ndarray]:
    """int32 params [P, target, len t1, len t2, len t3, infinite_resources] and tiers [3 x 40] for the
    engine / oracle."""
    params = np.array([config.num_players, config.target_points] + [len(t) for t in tiers0] +
                      [1 if config.infinite_resources else 0], dtype=np.int32)
    tiers = np.zeros((3, 40), dtype=np.int32)
    for t in range(3):
        tiers[t, :len(tiers0[t])] = tiers0[t]
    return params, np.ascontiguousarray(tiers.ravel())
