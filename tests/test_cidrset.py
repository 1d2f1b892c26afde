"""Node IPAM CIDR set (`pkg/controller/node/ipam/cidrset/cidr_set_test.go`)."""
import pytest

from kubernetes_amd.controllers.network import CIDRSet


@pytest.mark.parametrize("cluster,expected", [("127.123.234.0/30", "127.123.234.0/30"),
                                              ("beef:1234::/30", "beef:1234::/30")])
def test_fully_allocated(cluster, expected):
    s = CIDRSet(cluster, 30)
    assert s.allocate() == expected
    with pytest.raises(RuntimeError):
        s.allocate()
    s.release(expected)
    assert s.allocate() == expected


@pytest.mark.parametrize("cluster,mask", [("127.123.234.0/16", 24), ("beef:1234::/16", 24)])
def test_allocation_occupied(cluster, mask):
    s = CIDRSet(cluster, mask)
    cidrs = [s.allocate() for _ in range(256)]
    with pytest.raises(RuntimeError):
        s.allocate()
    for c in cidrs:
        s.release(c)
    for c in cidrs[128:]:
        s.occupy(c)
    again = [s.allocate() for _ in range(128)]
    with pytest.raises(RuntimeError):
        s.allocate()
    assert sorted(again) == sorted(cidrs[:128])


@pytest.mark.parametrize("cluster,mask,sub,begin,end", [
    ("127.0.0.0/8", 16, "127.0.0.0/8", 0, 255),
    ("2001:beef:1200::/40", 48, "2001:beef:1200::/40", 0, 255),
    ("127.0.0.0/8", 16, "127.0.0.0/2", 0, 255),
    ("2001:beef:1200::/40", 48, "2001:beef:1234::/34", 0, 255),
    ("127.0.0.0/8", 16, "127.0.0.0/16", 0, 0),
    ("127.0.0.0/8", 32, "127.0.0.0/16", 0, 65535),
    ("127.0.0.0/7", 16, "127.0.0.0/15", 256, 257),
    ("2001:beef:7f00::/39", 48, "2001:beef:7f00::/47", 256, 257),
    ("127.0.0.0/7", 15, "127.0.0.0/15", 128, 128),
])
def test_occupy(cluster, mask, sub, begin, end):
    """TestOccupy: the used range after occupying `sub`."""
    s = CIDRSet(cluster, mask)
    assert s.occupy(sub)
    assert (min(s.used), max(s.used), len(s.used)) == (begin, end, end - begin + 1)


def test_occupy_outside_the_cluster_range_fails():
    s = CIDRSet("10.0.0.0/16", 24)
    assert not s.occupy("192.168.0.0/24")
    assert not s.used


def test_ipv6_subnet_too_big():
    with pytest.raises(ValueError):
        CIDRSet("beef:1234::/30", 48)
