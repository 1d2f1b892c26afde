"""Cluster add-ons: DNS and the add-on manager (`cluster/addons`)."""
