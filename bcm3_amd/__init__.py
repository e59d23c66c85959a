"""bcm3_amd -- MI355X-native likelihood-evaluation hot path of BCM3."""
