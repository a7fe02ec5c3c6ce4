"""h264r -- MI355X-native H.264 macroblock reconstruction (host API)."""
