"""Command-line configuration with the reference's option names and parse
semantics (host side; the C shims in csrc/vp_nf_*.c do the same in C).

  vignat    vignat/nat_config.c:17-106   (--eth-dest --expire --extip
            --lan-dev --max-flows --starting-port --wan)
  vigbridge vigbridge/bridge_config.c:22-66 (--expire --capacity --config)
  viglb     viglb/lb_config.c:15-100     (--flow-expiration --flow-capacity
            --backend-capacity --cht-height --backend-expiration --wan)
  vigfw     vigfw/fw_config.c:17-82      (--eth-dest --expire --max-flows
            --wan)
  vigpol    vigpol/policer_config.c:17-93 (--lan --wan --rate --burst
            --capacity)

The reference calls exit(EXIT_FAILURE) on a bad option; here a ValueError is
raised with the same message.
"""
from __future__ import annotations

import re

from . import (BridgeConfigC, BridgeRuleC, FwConfigC, LbConfigC, NatConfigC,
               PolConfigC)


def _parse_int(s: str, name: str, nxt: str = "") -> tuple[int, str]:
    """nf_util_parse_int (nf-util.c:67-78): strtoimax base 10; the character
    after the number must be `nxt` ('' = end of string)."""
    m = re.match(r"\s*([+-]?\d+)", s)
    rest = s[m.end():] if m else s
    if not m or (rest[:1] != nxt if nxt else rest != ""):
        raise ValueError(f"Error while parsing '{name}': {s}")
    return int(m.group(1)), rest


def _parse_mac(s: str) -> bytes:
    """nf_parse_etheraddr (nf-parse.h:9-19): %02hhX:... six fields."""
    m = re.match(r"([0-9A-Fa-f]{1,2}):([0-9A-Fa-f]{1,2}):([0-9A-Fa-f]{1,2}):"
                 r"([0-9A-Fa-f]{1,2}):([0-9A-Fa-f]{1,2}):([0-9A-Fa-f]{1,2})", s)
    if not m:
        raise ValueError(f"Invalid MAC address: {s}")
    return bytes(int(x, 16) for x in m.groups())


def parse_ipv4(s: str) -> int:
    """nf_parse_ipv4addr (nf-parse.h:21-32): host-order a<<24|b<<16|c<<8|d
    (the value nat_main.c:96 stores raw into the header)."""
    m = re.match(r"(\d+)\.(\d+)\.(\d+)\.(\d+)", s)
    if not m:
        raise ValueError(f"Invalid external IP address: {s}")
    a, b, c, d = (int(x) & 0xFF for x in m.groups())
    return (a << 24) | (b << 16) | (c << 8) | d


def _split(argv):
    """getopt_long over `--name value` / `--name=value` pairs."""
    out = []
    i = 0
    while i < len(argv):
        a = argv[i]
        if not a.startswith("--"):
            raise ValueError("Unknown option.")
        if "=" in a:
            k, v = a[2:].split("=", 1)
        else:
            if i + 1 >= len(argv):
                raise ValueError(f"option '{a}' requires an argument")
            k, v = a[2:], argv[i + 1]
            i += 1
        out.append((k, v))
        i += 1
    return out


def nat_config_from_args(argv, n_devices: int, device_macs) -> NatConfigC:
    c = NatConfigC()
    c.n_devices = n_devices
    for d, m in enumerate(device_macs):  # rte_eth_macaddr_get
        c.device_macs[d][:] = list(m)
    for k, v in _split(argv):
        if k == "eth-dest":
            dev, _ = _parse_int(v, "eth-dest device", ",")
            if dev >= n_devices:
                raise ValueError(f"eth-dest: device {dev} >= nb_devices "
                                 f"({n_devices})")
            c.endpoint_macs[dev][:] = list(_parse_mac(v[2:]))
        elif k == "expire":
            c.expiration_time = _parse_int(v, "exp-time")[0] & 0xFFFFFFFF
            if c.expiration_time == 0:
                raise ValueError("Expiration time must be strictly positive.")
        elif k == "extip":
            c.external_addr = parse_ipv4(v)
        elif k == "lan-dev":
            c.lan_main_device = _parse_int(v, "lan-dev")[0] & 0xFFFF
            if c.lan_main_device >= n_devices:
                raise ValueError("Main LAN device does not exist.")
        elif k == "max-flows":
            c.max_flows = _parse_int(v, "max-flows")[0] & 0xFFFFFFFF
            if c.max_flows <= 0:
                raise ValueError("Flow table size must be strictly positive.")
        elif k == "starting-port":
            c.start_port = _parse_int(v, "start-port")[0] & 0xFFFF
        elif k == "wan":
            c.wan_device = _parse_int(v, "wan-dev")[0] & 0xFFFF
            if c.wan_device >= n_devices:
                raise ValueError("WAN device does not exist.")
        else:
            raise ValueError("Unknown option.")
    return c


def bridge_config_from_args(argv, n_devices: int, static_rules=()):
    """static_rules: (mac bytes, device_from, device_to) as read from the
    --config file by read_static_ft_from_file (bridge_main.c:130-230)."""
    c = BridgeConfigC()
    c.expiration_time = 300000000  # DEFAULT_EXP_TIME, bridge_config.c:14
    c.dyn_capacity = 128           # DEFAULT_CAPACITY, bridge_config.c:15
    c.n_devices = n_devices
    for k, v in _split(argv):
        if k == "expire":
            c.expiration_time = _parse_int(v, "exp-time")[0] & 0xFFFFFFFF
            if c.expiration_time <= 0:
                raise ValueError("Expiration time must be strictly positive.")
        elif k == "capacity":
            c.dyn_capacity = _parse_int(v, "capacity")[0] & 0xFFFFFFFF
            if c.dyn_capacity <= 0:
                raise ValueError("Flow table size must be strictly positive.")
        elif k == "config":
            static_rules = read_static_rules(v)
        else:
            raise ValueError(f"Unknown option {k}")
    rules = (BridgeRuleC * max(1, len(static_rules)))()
    for i, (mac, fr, to) in enumerate(static_rules):
        rules[i].mac[:] = list(mac)
        rules[i].device_from, rules[i].device_to = fr, to
    c.n_static = len(static_rules)
    c.static_rules = rules
    c._keep = rules
    return c


def read_static_rules(fname: str):
    """The --config file format of bridge_main.c:130-230: whitespace separated
    `MAC device_from device_to` triples."""
    toks = open(fname).read().split()
    rules = []
    for i in range(0, len(toks) - 2, 3):
        try:
            rules.append((_parse_mac(toks[i]), int(toks[i + 1]),
                          int(toks[i + 2])))
        except ValueError:
            continue
    return rules


def lb_config_from_args(argv, n_devices: int, device_macs) -> LbConfigC:
    c = LbConfigC()
    c.n_devices = n_devices
    for d, m in enumerate(device_macs):
        c.device_macs[d][:] = list(m)
    for k, v in _split(argv):
        val = _parse_int(v, k)[0] & 0xFFFFFFFF
        if k == "flow-expiration":
            c.flow_expiration_time = val
        elif k == "flow-capacity":
            c.flow_capacity = val
        elif k == "backend-capacity":
            c.backend_capacity = val
        elif k == "cht-height":
            c.cht_height = val
        elif k == "backend-expiration":
            c.backend_expiration_time = val
        elif k == "wan":
            c.wan_device = val & 0xFFFF
            if c.wan_device >= n_devices:
                raise ValueError("WAN device does not exist.")
        else:
            raise ValueError("Unknown option.")
        if val == 0 and k != "wan":
            raise ValueError(f"{k} must be strictly positive.")
    return c


def fw_config_from_args(argv, n_devices: int, device_macs) -> FwConfigC:
    c = FwConfigC()
    c.n_devices = n_devices
    for d, m in enumerate(device_macs):  # rte_eth_macaddr_get
        c.device_macs[d][:] = list(m)
    for k, v in _split(argv):
        if k == "eth-dest":
            dev, _ = _parse_int(v, "eth-dest device", ",")
            if dev >= n_devices:
                raise ValueError(f"eth-dest: device {dev} >= nb_devices "
                                 f"({n_devices})")
            c.endpoint_macs[dev][:] = list(_parse_mac(v[2:]))
        elif k == "expire":
            c.expiration_time = _parse_int(v, "exp-time")[0] & 0xFFFFFFFF
            if c.expiration_time == 0:
                raise ValueError("Expiration time must be strictly positive.")
        elif k == "max-flows":
            c.max_flows = _parse_int(v, "max-flows")[0] & 0xFFFFFFFF
            if c.max_flows <= 0:
                raise ValueError("Flow table size must be strictly positive.")
        elif k == "wan":
            c.wan_device = _parse_int(v, "wan-dev")[0] & 0xFFFF
            if c.wan_device >= n_devices:
                raise ValueError("WAN device does not exist.")
        else:
            raise ValueError("Unknown option.")
    return c


def pol_config_from_args(argv, n_devices: int) -> PolConfigC:
    """policer_config.c:17-93: defaults LAN 1, WAN 0, rate 1 MB/s, burst
    100 kB, capacity 128; devices must exist, rate/burst/capacity > 0."""
    c = PolConfigC()
    c.n_devices = n_devices
    c.lan_device, c.wan_device = 1, 0
    c.rate, c.burst, c.dyn_capacity = 1_000_000, 100_000, 128
    for k, v in _split(argv):
        if k == "lan":
            c.lan_device = _parse_int(v, "lan")[0] & 0xFFFF
            if c.lan_device >= n_devices:
                raise ValueError("Invalid LAN device.")
        elif k == "wan":
            c.wan_device = _parse_int(v, "wan")[0] & 0xFFFF
            if c.wan_device >= n_devices:
                raise ValueError("Invalid WAN device.")
        elif k == "rate":
            c.rate = _parse_int(v, "rate")[0] & 0xFFFFFFFFFFFFFFFF
            if c.rate == 0:
                raise ValueError("Policer rate must be strictly positive.")
        elif k == "burst":
            c.burst = _parse_int(v, "burst")[0] & 0xFFFFFFFFFFFFFFFF
            if c.burst == 0:
                raise ValueError("Policer burst size must be strictly positive.")
        elif k == "capacity":
            c.dyn_capacity = _parse_int(v, "capacity")[0] & 0xFFFFFFFF
            if c.dyn_capacity <= 0:
                raise ValueError("Flow table size must be strictly positive.")
        else:
            raise ValueError("Unknown option.")
    return c
