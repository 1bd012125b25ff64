"""A real TPACKET_V3 PACKET_RX_RING on the loopback device, set up the way
netsniff-ng's RX path does (ring_rx.c:28-229: setup_rx_ring_layout with
tpacket_req3, PACKET_VERSION TPACKET_V3, PACKET_RX_RING, mmap of
block_size * block_nr, bind to the device), with frames sent into it from
a second AF_PACKET socket.  Needs CAP_NET_RAW: open() raises
PermissionError without it (the tests skip).  Test infrastructure."""
import mmap
import select
import socket
import struct
import time

import numpy as np

SOL_PACKET = 263
PACKET_RX_RING = 5
PACKET_VERSION = 10
TPACKET_V3 = 2
ETH_P_ALL = 0x0003
TP_STATUS_KERNEL, TP_STATUS_USER = 0, 1


class Ring:
    def __init__(self, block_size=1 << 22, block_nr=4, frame_size=1 << 11, tov_ms=20, dev="lo"):
        self.sock = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(ETH_P_ALL))
        try:
            self.sock.setsockopt(SOL_PACKET, PACKET_VERSION, TPACKET_V3)
            req = struct.pack("7I", block_size, block_nr, frame_size, block_size * block_nr // frame_size,
                              tov_ms, 0, 0)
            self.sock.setsockopt(SOL_PACKET, PACKET_RX_RING, req)
            self.size = block_size * block_nr
            self.map = mmap.mmap(self.sock.fileno(), self.size, mmap.MAP_SHARED,
                                 mmap.PROT_READ | mmap.PROT_WRITE)
            self.sock.bind((dev, ETH_P_ALL))
        except Exception:
            self.sock.close()
            raise
        self.block_size, self.block_nr = block_size, block_nr
        self.ifindex = socket.if_nametoindex(dev)
        self.dev = dev
        self.next = 0

    def send(self, frames):
        tx = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, 0)
        try:
            tx.bind((self.dev, 0))
            for f in frames:
                tx.send(f)
        finally:
            tx.close()

    def block(self, k):
        """Block k of the ring as a uint8 array over the mapping (no copy)."""
        return np.frombuffer(self.map, dtype=np.uint8, count=self.block_size, offset=k * self.block_size)

    def status(self, k):
        return struct.unpack_from("<I", self.map, k * self.block_size + 8)[0]

    def wait_block(self, timeout=5.0):
        """The next retired block (TP_STATUS_USER), in ring order, or None."""
        k = self.next
        end = time.time() + timeout
        while not self.status(k) & TP_STATUS_USER:
            left = end - time.time()
            if left <= 0:
                return None
            select.select([self.sock], [], [], min(left, 0.05))
        self.next = (k + 1) % self.block_nr
        return k

    def release(self, k):
        """Hand block k back to the kernel (flush_block, ring_rx.c)."""
        struct.pack_into("<I", self.map, k * self.block_size + 8, TP_STATUS_KERNEL)

    def close(self):
        try:
            self.map.close()
        except BufferError:
            pass           # arrays over the mapping still alive: it closes with them
        self.sock.close()


def open_ring(**kw):
    """A Ring, or None when the process may not open packet sockets."""
    import errno
    try:
        return Ring(**kw)
    except PermissionError:
        return None
    except OSError as e:
        if e.errno in (errno.EPERM, errno.EACCES, errno.EAFNOSUPPORT, errno.ENODEV):
            return None
        raise


MARK = bytes.fromhex("026e73640001")


def marked(frames):
    """Frames with the test's source MAC (to tell them from other lo traffic)."""
    return [f[:6] + MARK + f[12:] for f in frames if len(f) >= 14]


def collect(ring, want, blocks_cb, timeout=10.0):
    """Retired blocks until `want` marked frames came through; blocks_cb(k)
    returns the block's kept frames (bytes) and is called before release."""
    got = []
    end = time.time() + timeout
    while len(got) < want and time.time() < end:
        k = ring.wait_block(max(0.1, end - time.time()))
        if k is None:
            break
        got += [f for f in blocks_cb(k) if f[6:12] == MARK]
        ring.release(k)
    return got
