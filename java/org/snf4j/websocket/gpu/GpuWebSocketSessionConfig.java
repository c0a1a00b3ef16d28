/*
 * The install hook: a DefaultWebSocketSessionConfig whose switchDecoders /
 * switchEncoders (IWebSocketSessionConfig.java:123,133; default
 * DefaultWebSocketSessionConfig.java:271-281) put the MI355X codec under the
 * reference's keys, so extensions that addAfter("ws-decoder" | "ws-encoder")
 * (PerMessageDeflateExtension.java:303-326) still find them.
 *
 * UTF-8 validation is fused into the device decode unless extensions are allowed:
 * with permessage-deflate the text must be validated after inflate
 * (PerMessageDeflateExtension.java:316-326), so the decode runs with the fused
 * check off and the reference's FrameUtf8Validator stays at "ws-utf8-validator"
 * behind the extension's decoder.
 */
package org.snf4j.websocket.gpu;

import java.net.URI;

import org.snf4j.core.codec.ICodecPipeline;
import org.snf4j.websocket.DefaultWebSocketSessionConfig;
import org.snf4j.websocket.frame.FrameUtf8Validator;

public class GpuWebSocketSessionConfig extends DefaultWebSocketSessionConfig {

	private final WsgBatcher batcher;
	private int encodeThreshold = 1 << 20;

	/** Client mode (the request URI is given), as DefaultWebSocketSessionConfig(URI). */
	public GpuWebSocketSessionConfig(URI requestUri, WsgBatcher batcher) {
		super(requestUri);
		this.batcher = batcher;
	}

	/** Server mode, as DefaultWebSocketSessionConfig(). */
	public GpuWebSocketSessionConfig(WsgBatcher batcher) {
		super();
		this.batcher = batcher;
	}

	/** Payload bytes from which a frame is encoded on the device (smaller: on the loop thread). */
	public GpuWebSocketSessionConfig setEncodeThreshold(int bytes) {
		encodeThreshold = bytes;
		return this;
	}

	@Override
	public void switchEncoders(ICodecPipeline pipeline, boolean allowExtensions) {
		pipeline.replace(HANDSHAKE_ENCODER, WEBSOCKET_ENCODER,
				new GpuFrameEncoder(isClientMode(), batcher, encodeThreshold));
	}

	@Override
	public void switchDecoders(ICodecPipeline pipeline, boolean allowExtensions) {
		boolean fused = !allowExtensions;
		pipeline.replace(HANDSHAKE_DECODER, WEBSOCKET_DECODER,
				new GpuFrameDecoder(isClientMode(), allowExtensions, getMaxFramePayloadLength(), fused, batcher));
		if (!fused)
			pipeline.addAfter(WEBSOCKET_DECODER, WEBSOCKET_UTF8_VALIDATOR, new FrameUtf8Validator());
	}
}
