"""onet wire format: dedis/protobuf codec, message envelopes, struct converters."""
