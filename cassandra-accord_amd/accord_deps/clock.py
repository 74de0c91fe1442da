"""The node clock part of PreAccept's witnessedAt, host side.

`ad_preaccept_device` (include/accord_deps.h) returns, per request, what CommandStore.preaccept
(CommandStore.java:322-347) derives from the store: minNonConflicting (maxConflicts over the keys)
and the AD_PA_* decision. The Timestamp it answers with also needs the node's clock, which lives on
the host: Node.uniqueNow / uniqueNow(atLeast) (Node.java:348-389) over the node's `now` Timestamp.
This module restates that clock so a host composes the reference's witnessedAt exactly:

    FAST      -> txnId
    REJECTED  -> uniqueNow(txnId).asRejected()
    ESP       -> txnId                                 (ExclusiveSyncPoint, :333-337)
    otherwise -> uniqueNow(minNonConflicting)

Timestamps are (msb, lsb, node) triples in the reference's bit layout (Timestamp.java:81-88):
msb = epoch << 15 | hlc >> 48 (15 high hlc bits), lsb = (hlc << 16) | flags.
"""
REJECTED_FLAG = 0x8000          # Timestamp.java:32
IDENTITY_FLAGS = 0x001E         # Timestamp.java:42
MASK64 = (1 << 64) - 1

AD_PA_FAST, AD_PA_REJECTED, AD_PA_ESP = 1, 2, 4


def epoch_of(t):
    return t[0] >> 15


def hlc_of(t):
    return ((t[0] & 0x7FFF) << 48) | (t[1] >> 16)


def flags_of(t):
    return t[1] & 0xFFFF


def make(epoch, hlc, flags, node):
    """Timestamp.fromValues(epoch, hlc, flags, node)."""
    return ((epoch << 15) | (hlc >> 48)) & MASK64, ((hlc << 16) | flags) & MASK64, int(node)


def compare(a, b):
    """Timestamp.compareTo (Timestamp.java:209-217): msb unsigned, low hlc bits, identity flags, node."""
    for x, y in ((a[0], b[0]), (a[1] >> 16, b[1] >> 16), (a[1] & IDENTITY_FLAGS, b[1] & IDENTITY_FLAGS), (a[2], b[2])):
        if x != y:
            return -1 if x < y else 1
    return 0


class NodeClock:
    """Node.now with uniqueNow / uniqueNow(atLeast) (Node.java:348-389). `now_hlc` is the hlc the
    node's clock supplier returns; it is read on every uniqueNow (set_time / advance move it)."""

    def __init__(self, node_id, now_hlc, epoch=0):
        # Node's constructor: Timestamp.fromValues(topology.epoch(), nowSupplier.getAsLong(), id)
        self.node = int(node_id)
        self.clock = int(now_hlc)
        self.topology_epoch = int(epoch)
        self.now = make(epoch, now_hlc, 0, node_id)

    def advance(self, by):
        self.clock += int(by)

    def set_epoch(self, epoch):
        """The topology learned a new epoch (ConfigurationService reportTopology)."""
        self.topology_epoch = max(self.topology_epoch, int(epoch))

    def unique_now(self, at_least=None):
        if at_least is not None and compare(self.now, at_least) < 0:
            self.now = self._now_at_least(self.now, at_least)
        cur = self.now
        # cur.withNextHlc(nowSupplier).withEpochAtLeast(topology.epoch())
        nxt = make(epoch_of(cur), max(self.clock, hlc_of(cur) + 1), flags_of(cur), cur[2])
        if self.topology_epoch > epoch_of(nxt):
            nxt = make(self.topology_epoch, hlc_of(nxt), flags_of(nxt), nxt[2])
        self.now = nxt
        return nxt

    @staticmethod
    def _now_at_least(current, proposed):
        # Node.nowAtLeast: current if it is at least proposed in epoch and hlc, else proposed lifted
        # to current's hlc with current's node (flags of proposed kept)
        if epoch_of(current) >= epoch_of(proposed) and hlc_of(current) >= hlc_of(proposed):
            return current
        hlc = max(hlc_of(proposed), hlc_of(current))
        return make(epoch_of(proposed), hlc, flags_of(proposed), current[2])

    def witnessed_at(self, txn_id, min_non_conflicting, pa_flags):
        """The Timestamp CommandStore.preaccept returns for one request, given the store-side answer
        of ad_preaccept_device (minNonConflicting, AD_PA_* flags)."""
        txn_id = tuple(int(x) for x in txn_id)
        if pa_flags & AD_PA_REJECTED:
            t = self.unique_now(txn_id)
            return t[0], t[1] | REJECTED_FLAG, t[2]
        if pa_flags & (AD_PA_FAST | AD_PA_ESP):
            return txn_id
        return self.unique_now(tuple(int(x) for x in min_non_conflicting))

    def witnessed_at_batch(self, txns, min_nc, pa_flags):
        """witnessed_at over a batch in request order (the clock advances as the reference's does when
        the node processes the requests one after another). Tids in, list of triples out."""
        return [self.witnessed_at((int(txns.msb[i]), int(txns.lsb[i]), int(txns.node[i])),
                                  (int(min_nc.msb[i]), int(min_nc.lsb[i]), int(min_nc.node[i])), int(pa_flags[i]))
                for i in range(len(pa_flags))]
