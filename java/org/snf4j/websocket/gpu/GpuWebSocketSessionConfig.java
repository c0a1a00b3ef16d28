/*
 * The install hook: a DefaultWebSocketSessionConfig whose switchDecoders /
 * switchEncoders (IWebSocketSessionConfig.java:123,133; default
 * DefaultWebSocketSessionConfig.java:271-281) put the MI355X codec under the
 * reference's keys, so extensions that addAfter("ws-decoder" | "ws-encoder")
 * (PerMessageDeflateExtension.java:303-326) still find them:
 *   "ws-decoder"        GpuFrameDecoder (FrameDecoder)
 *   "ws-utf8-validator" GpuFrameUtf8Validator (FrameUtf8Validator), as the reference
 *                       always adds it; directly behind the decoder it is the check
 *                       fused into the decode kernels, behind GPU inflate it is the
 *                       validator stage of the same batch
 *   "ws-aggregator"     GpuFrameAggregator, if setAggregation() asked for one
 *   "ws-encoder"        GpuFrameEncoder (FrameEncoder)
 * permessage-deflate with the GPU inflate: list GpuPerMessageDeflateExtension in
 * getSupportedExtensions().  The batcher serves the loop the sessions belong to.
 */
package org.snf4j.websocket.gpu;

import java.net.URI;

import org.snf4j.core.codec.ICodecPipeline;
import org.snf4j.websocket.DefaultWebSocketSessionConfig;

public class GpuWebSocketSessionConfig extends DefaultWebSocketSessionConfig {

	private final WsgBatcher batcher;
	private int encodeThreshold = GpuFrameEncoder.DEFAULT_DEVICE_THRESHOLD;
	private int maxAggregatedLength = -1;

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

	/** Aggregate fragmented messages (FrameAggregator(maxAggregatedLength)) in the device batch. */
	public GpuWebSocketSessionConfig setAggregation(int maxAggregatedLength) {
		this.maxAggregatedLength = maxAggregatedLength;
		return this;
	}

	@Override
	public void switchEncoders(ICodecPipeline pipeline, boolean allowExtensions) {
		pipeline.replace(HANDSHAKE_ENCODER, WEBSOCKET_ENCODER,
				new GpuFrameEncoder(isClientMode(), batcher, encodeThreshold));
	}

	@Override
	public void switchDecoders(ICodecPipeline pipeline, boolean allowExtensions) {
		pipeline.replace(HANDSHAKE_DECODER, WEBSOCKET_DECODER,
				new GpuFrameDecoder(isClientMode(), allowExtensions, getMaxFramePayloadLength(), batcher));
		pipeline.addAfter(WEBSOCKET_DECODER, WEBSOCKET_UTF8_VALIDATOR, new GpuFrameUtf8Validator());
		if (maxAggregatedLength >= 0)
			pipeline.addAfter(WEBSOCKET_UTF8_VALIDATOR, GpuFrameAggregator.KEY,
					new GpuFrameAggregator(maxAggregatedLength));
	}
}
