"""Typed map wrappers mirroring Cilium's pkg/maps/* key/value layouts."""
